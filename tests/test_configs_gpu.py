"""GPU parity at the benchmark configurations' real shapes (BASELINE.json
configs 2-4), bit-exact against the oracle:

  cfg2  mixed MTU {64, 256, 1500, 9000} B packets (CT {12, 204, 1448, 8948} B)
        over 1024 AES-128-GCM SAs, random SA per record, through the device
        planner (ungrouped descriptors), driver SA table of 2048 slots;
  cfg3  1496-B packets (1440-B CT) over 1024 AES-256-CBC + HMAC-SHA1-96 SAs;
  cfg4  rank 0 of 8: the packets and SAs shard_plan gives rank 0 of a global
        batch over 8192 random SPIs (fnv_32 SPI hash, key.c:295-299).

Record counts are the full SA count and >= 64K records per configuration
(per rank for cfg4); the oracle checks every record.  cfg1 at its full size
(1M records) is checked record by record in test_gcm_gpu.py, cfg2-4 in
test_configs_full_gpu.py."""
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
    d = GpuCryptoDriver(max_sessions=2048)
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
            sa = SecAssoc(s.spi, GCM, s.key + s.salt, esn=s.esn, mlen=s.mlen)
        rc, sid = drv.newsession(sa.csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
    return np.array(sids)


def _payload_mask(descs, size, hlen, alen):
    """Vectorised: True over every record's payload bytes."""
    starts = descs["off4"].astype(np.int64) * 4 + hlen
    ends = descs["off4"].astype(np.int64) * 4 + descs["len"].astype(np.int64) - alen
    edge = np.zeros(size + 1, dtype=np.int32)
    np.add.at(edge, starts, 1)
    np.add.at(edge, ends, -1)
    return np.cumsum(edge[:-1]) > 0


def _flip_icvs(rng, ct, descs, frac, alen):
    bad = ct.copy()
    flip = rng.random(len(descs)) < frac
    for i in np.nonzero(flip)[0]:
        bad[int(descs["off4"][i]) * 4 + int(descs["len"][i]) - 1 - int(rng.integers(0, alen))] ^= 0x08
    return bad, flip


def _check_decrypt(drv, sids, sa_idx, descs, bad, flip, ref_out, ref_st, plain, hlen, alen):
    from espgpu.batch import decrypt_batch
    n = len(descs)
    d = descs.copy()
    d["sa"] = sids[sa_idx]
    ok_mask = _payload_mask(descs[~flip], len(bad), hlen, alen)
    assert (ref_out[ok_mask] == plain[ok_mask]).all()
    for inplace in (False, True):
        arena = _dev(bad)
        out = arena if inplace else torch.zeros_like(arena)
        st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
        decrypt_batch(drv, arena, _descs_dev(d), n, st, out=None if inplace else out, grouped=False)
        torch.cuda.synchronize()
        got = st.cpu().numpy()
        assert (got == ref_st).all(), (inplace, np.nonzero(got != ref_st)[0][:10])
        res = out.cpu().numpy()
        assert (res[ok_mask] == ref_out[ok_mask]).all()
        if inplace:      # verify-first: failed records keep their ciphertext
            bad_mask = _payload_mask(descs[flip], len(bad), hlen, alen)
            assert (res[bad_mask] == bad[bad_mask]).all()
        del arena, out


def test_cfg2_mixed_mtu_1k_gcm_sas(drv):
    rng = np.random.default_rng(0xC2)
    nsa, n = 1024, 1 << 16
    sas = [GcmSA(rng, 16) for _ in range(nsa)]
    sids = _sessions(drv, sas)
    sa_idx = rng.integers(0, nsa, n)
    cts = rng.choice([12, 204, 1448, 8948], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts)
    assert len(np.unique(sa_idx)) == nsa
    bad, flip = _flip_icvs(rng, ct, descs, 0.01, 16)
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    _check_decrypt(drv, sids, sa_idx, descs, bad, flip, ref_out, ref_st, plain, 16, 16)
    # encrypt direction at the same shape: CT and ICVs bit-exact
    from espgpu.batch import encrypt_batch
    d = descs.copy()
    d["sa"] = sids[sa_idx]
    arena = _dev(plain)
    st = torch.full((n,), 0xEE, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, _descs_dev(d), n, st, grouped=False)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == 0).all()
    assert (arena.cpu().numpy() == ct).all()
    for s in sids:
        drv.freesession(int(s))


def test_cfg3_1k_eta_sas(drv):
    rng = np.random.default_rng(0xC3)
    nsa, n = 1024, 1 << 16
    sas = [EtaSA(rng, 32) for _ in range(nsa)]
    sids = _sessions(drv, sas)
    sa_idx = rng.integers(0, nsa, n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, np.full(n, 1440), gcm=False)
    bad, flip = _flip_icvs(rng, ct, descs, 0.01, 12)
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    _check_decrypt(drv, sids, sa_idx, descs, bad, flip, ref_out, ref_st, plain, 24, 12)
    for s in sids:
        drv.freesession(int(s))


@pytest.mark.parametrize("rank", range(8))
def test_cfg4_rank_of_8_spi_shard(drv, rank):
    """cfg4's per-GPU workload for every rank of an 8-GPU job: the rank's
    ~1K SAs of 8192 random SPIs (fnv1_32(spi) mod 8, key.c:295) and their
    packets, decrypted through the planner on this one GPU vs the oracle."""
    from espgpu.shard import gpu_of_spi, random_spis, shard_plan
    world, nsa_glob, n_glob = 8, 8192, 8 * 72000
    spis = random_spis(nsa_glob, 0xC4)
    sa_glob = np.random.default_rng(0xC40).integers(0, nsa_glob, n_glob)
    local_sas, local_pkts = shard_plan(spis, sa_glob, rank, world)
    assert 900 < len(local_sas) < 1150 and all(gpu_of_spi(spis[i], world) == rank for i in local_sas)
    assert len(local_pkts) >= 1 << 16
    remap = np.full(nsa_glob, -1, dtype=np.int64)
    remap[local_sas] = np.arange(len(local_sas))
    sa_idx = remap[sa_glob[local_pkts]]
    assert (sa_idx >= 0).all()
    rng = np.random.default_rng(0xC41 + rank)
    sas = [GcmSA(rng, 16, spi=int(spis[i])) for i in local_sas]
    sids = _sessions(drv, sas)
    n = len(local_pkts)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, np.full(n, 1448))
    bad, flip = _flip_icvs(rng, ct, descs, 0.01, 16)
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    _check_decrypt(drv, sids, sa_idx, descs, bad, flip, ref_out, ref_st, plain, 16, 16)
    for s in sids:
        drv.freesession(int(s))


def test_planner_runs_of_one_session(drv):
    """Planner batch whose sessions hold hundreds of chunks each (4 GCM SAs x
    ~200K records of two size classes, so a workgroup's consecutive tickets
    are mostly of one session and it restages only on a change); every
    record against the oracle, out of place and in place."""
    rng = np.random.default_rng(0xC5)
    nsa, n = 4, 800_000
    sas = [GcmSA(rng, 16) for _ in range(nsa)]
    sids = _sessions(drv, sas)
    sa_idx = rng.integers(0, nsa, n)
    cts = rng.choice([12, 204], n)
    plain, ct, descs, eh = build_records(rng, sas, sa_idx, cts)
    bad, flip = _flip_icvs(rng, ct, descs, 0.01, 16)
    ref_out, ref_st = oracle_decrypt(sas, bad, descs, eh)
    assert (ref_st[flip] == O.EBADMSG).all() and (ref_st[~flip] == 0).all()
    _check_decrypt(drv, sids, sa_idx, descs, bad, flip, ref_out, ref_st, plain, 16, 16)
    for s in sids:
        drv.freesession(int(s))
