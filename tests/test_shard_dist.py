"""SPI-hash sharding and the bench's N>1 reduction, on CPU.

world_size-2 `gloo` runs exercise the same code bench.py runs under torchrun
with RCCL: each rank plans its share of one global batch, the shares must
partition the batch, and the reported value uses sum-of-bytes / max-of-time.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from espgpu.shard import fnv_32_buf, gpu_of_spi, key_u32hash, random_spis, shard_plan, spis_for_rank  # noqa: E402

SMALL_CFG4 = dict(workload="cfg4-small", packets=4096, pkt=1500, skip=20, klen=16, nsa=64,
                  mixed=False, alg="gcm", sharded=True)


def test_fnv1_32_known_values():
    # FNV-1 32 (multiply then xor) with FreeBSD's FNV1_32_INIT, fnv_hash.h:23-31
    assert fnv_32_buf(b"") == 33554467
    h = 33554467
    for b in b"\x00\x00\x01\x00":
        h = (h * 0x01000193) & 0xFFFFFFFF
        h ^= b
    assert key_u32hash(0x100) == h


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_plan_partitions_batch(world):
    spis = random_spis(256, 7)
    assert len(set(spis)) == 256 and min(spis) >= 256
    sa_of = np.random.default_rng(1).integers(0, 256, 20000)
    seen_p, seen_s = [], []
    for r in range(world):
        sas, pk = shard_plan(spis, sa_of, r, world)
        assert all(gpu_of_spi(spis[i], world) == r for i in sas)
        assert all(gpu_of_spi(spis[sa_of[p]], world) == r for p in pk[:500])
        seen_p.append(pk)
        seen_s.append(sas)
    allp = np.concatenate(seen_p)
    assert len(allp) == len(sa_of) and len(np.unique(allp)) == len(sa_of)
    assert len(np.unique(np.concatenate(seen_s))) == 256
    if world > 1:   # balance within a loose bound for 256 random SPIs
        counts = np.array([len(p) for p in seen_p])
        assert counts.min() > 0.5 * counts.mean()


def test_spis_for_rank_disjoint():
    a, b = spis_for_rank(0, 2, 100), spis_for_rank(1, 2, 100)
    assert not set(a) & set(b)
    assert all(gpu_of_spi(s, 2) == 0 for s in a) and all(gpu_of_spi(s, 2) == 1 for s in b)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "f-stack_amd"))
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(0xE5B00001 + rank)
        spis, sa_of, sizes = bench.plan_packets(SMALL_CFG4, rank, world, rng)
        assert all(gpu_of_spi(s, world) == rank for s in spis)
        assert sa_of.min() >= 0 and sa_of.max() < len(spis)
        nbytes = int(sizes.sum())
        dt = 0.5 + rank                      # rank 1 is the slow one
        mdt, total = bench.aggregate(dist, world, dt, nbytes, torch.device("cpu"))
        got = [None] * world
        dist.all_gather_object(got, (sorted(spis), len(sizes)))
        counts = bench.per_rank(dist, world, rank, len(sizes), torch.device("cpu"))
        assert counts == [g[1] for g in got]
        # in-place copies: every rank takes the smallest count (equal segments)
        assert bench.agree_min(dist, world, 20 - 7 * rank, torch.device("cpu")) == 13
        q.put((rank, mdt, total, nbytes, got))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_bench_plan():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    totals = {r[2] for r in res}
    assert len(totals) == 1
    assert totals.pop() == sum(r[3] for r in res)        # sum of bytes over ranks
    assert all(abs(r[1] - 1.5) < 1e-9 for r in res)      # max of time over ranks
    spis0, n0 = res[0][4][0]
    spis1, n1 = res[0][4][1]
    assert not set(spis0) & set(spis1)
    assert len(spis0) + len(spis1) == SMALL_CFG4["nsa"] * world
    assert n0 + n1 == SMALL_CFG4["packets"] * world
