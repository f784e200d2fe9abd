#!/usr/bin/env python3
"""Benchmark: device-resident ESP AES-128-GCM decrypt, 1M x 1500-B packets per GPU.

One step = one pass of the hot path (verify + decrypt) over one batch of
1,048,576 ESP records already resident in HBM (BASELINE.json configs[1]).
N GPUs = N processes (torchrun), each with its own SAs chosen so that
fnv1_32(spi) mod N == rank (SPI-hash sharding, no collective on the data path);
per-GPU work is fixed (weak scaling) and value = all ranks' bytes / max time.

Prints ONE JSON line (rank 0) with the metric, a roofline object for the
dominant kernel (algorithmic bytes / HIP-event time on the launch stream) and a
cpu_baseline object (the oracle's cryptosoft-shaped restatement, timed on this
host's cores on a bounded sample of the same records).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "f-stack_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CONFIGS = {
    "cfg0": dict(workload="cfg0: 64K x 64B ESP AES-128-GCM decrypt, single SA", packets=1 << 16,
                 pkt=64, skip=20, klen=16, nsa=1, mixed=False, alg="gcm"),
    "cfg1": dict(workload="cfg1: 1M x 1500B ESP AES-128-GCM decrypt, single SA", packets=1 << 20,
                 pkt=1500, skip=20, klen=16, nsa=1, mixed=False, alg="gcm"),
    "cfg2": dict(workload="cfg2: 1M x {64,256,1500,9000}B mixed-MTU ESP AES-128-GCM decrypt, 1K SAs",
                 packets=1 << 20, pkt=None, skip=20, klen=16, nsa=1024, mixed=True, alg="gcm"),
    "cfg3": dict(workload="cfg3: 1M x 1496B ESP AES-256-CBC + HMAC-SHA1-96 decrypt, 1K SAs",
                 packets=1 << 20, pkt=1496, skip=20, klen=32, nsa=1024, mixed=False, alg="eta"),
    "cfg4": dict(workload="cfg4: N x 1M x 1500B ESP AES-128-GCM decrypt, N x 1K random SPIs, "
                          "packets routed to GPU fnv1_32(spi) mod N",
                 packets=1 << 20, pkt=1500, skip=20, klen=16, nsa=1024, mixed=False, alg="gcm",
                 sharded=True),
}
HDR_TRAILER = {"gcm": 8 + 8 + 16, "eta": 8 + 16 + 12}     # SPI|SN + IV + ICV per record


def aggregate(dist, world, dt, nbytes, device):
    """Max wall time and summed bytes over ranks (value = sum bytes / max time)."""
    if world == 1:
        return dt, nbytes
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    b = torch.tensor([float(nbytes)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    return float(t.item()), int(b.item())


def per_rank(dist, world, rank, value, device):
    """[value of rank 0, ..., value of rank world-1] (one all_reduce)."""
    if world == 1:
        return [value]
    import torch
    t = torch.zeros(world, dtype=torch.float64, device=device)
    t[rank] = float(value)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [int(x) for x in t.tolist()]


def hbm_copy_gbs(arena, reps=5):
    """Measured device-to-device copy rate over the same arena (bytes read +
    written / time): the practical HBM ceiling beside the 8 TB/s spec peak."""
    import torch
    dst = torch.empty_like(arena)
    dst.copy_(arena)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(arena)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del dst
    return 2 * arena.numel() / (ms * 1e-3) / 1e9


def plan_packets(cfg, rank, world, rng):
    """(spis, sa_of_packet, sizes) of the records this rank processes.

    cfg1-3: every rank owns `nsa` SAs whose SPI hashes to it (weak scaling).
    cfg4: one global batch of N x 1M packets over N x 1K random SPIs; each rank
    keeps the packets whose SA hashes to it (fnv1_32(spi) mod N, key.c:295)."""
    from espgpu.shard import random_spis, shard_plan, spis_for_rank
    if cfg.get("sharded"):
        nsa_glob, n_glob = cfg["nsa"] * world, cfg["packets"] * world
        spis_glob = random_spis(nsa_glob, 0xE5B00004)
        grng = np.random.default_rng(0xE5B00005)
        sa_glob = grng.integers(0, nsa_glob, n_glob)
        local_sas, local_pkts = shard_plan(spis_glob, sa_glob, rank, world)
        remap = np.full(nsa_glob, -1, dtype=np.int64)
        remap[local_sas] = np.arange(len(local_sas))
        sa_of = remap[sa_glob[local_pkts]]
        return [spis_glob[i] for i in local_sas], sa_of, np.full(len(local_pkts), cfg["pkt"])
    n = cfg["packets"]
    spis = spis_for_rank(rank, world, cfg["nsa"])
    if cfg["mixed"]:
        sizes = rng.choice(np.array([64, 256, 1500, 9000]), n)
    else:
        sizes = np.full(n, cfg["pkt"])
    sa_of = rng.integers(0, cfg["nsa"], n) if cfg["nsa"] > 1 else np.zeros(n, dtype=np.int64)
    return spis, sa_of, sizes


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg1", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = min(16, cores available)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--inplace", action="store_true", help="verify-first in-place decrypt")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive host-to-host leg")
    ap.add_argument("--e2e-chunk", type=int, default=65536, help="records per pipelined step")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from espgpu.batch import decrypt_batch, encrypt_batch
    from espgpu.esp import CBC_SHA1, GCM, SecAssoc
    from espgpu.opencrypto import GpuCryptoDriver

    cfg = CONFIGS[args.config]
    rng = np.random.default_rng(0xE5B00001 + rank)
    spis, sa_of, sizes = plan_packets(cfg, rank, world, rng)
    n = len(sizes)
    drv = GpuCryptoDriver(device=local, max_sessions=max(16, len(spis) + 8))
    sids, salts, keys = [], [], []
    for spi in spis:
        if cfg["alg"] == "gcm":
            key = rng.integers(0, 256, cfg["klen"] + 4, dtype=np.uint8).tobytes()
            sa = SecAssoc(spi, GCM, key)
            salts.append(int.from_bytes(key[-4:], "little"))
        else:
            key = (rng.integers(0, 256, cfg["klen"], dtype=np.uint8).tobytes(),
                   rng.integers(0, 256, 20, dtype=np.uint8).tobytes())
            sa = SecAssoc(spi, CBC_SHA1, key[0], key[1])
            salts.append(0)
        keys.append(key)
        rc, sid = drv.newsession(sa.csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)

    # ---- synthetic records, laid out as packet slots (outer IPv4 header at 0) ----
    slot = (sizes + 3) & ~3
    offs = np.concatenate([[0], np.cumsum(slot)[:-1]])
    total = int(slot.sum()) + 64
    d = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")])
    d["off4"] = (offs + cfg["skip"]) // 4
    d["len"] = sizes - cfg["skip"]
    d["sa"] = np.array(sids)[sa_of]
    d["salt"] = np.array(salts, dtype=np.uint32)[sa_of]
    desc = torch.from_numpy(d.view(np.uint8).copy()).to(dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    arena = torch.randint(0, 256, (total,), dtype=torch.uint8, device=dev, generator=g)
    status = torch.zeros(n, dtype=torch.uint8, device=dev)
    grouped = len(spis) == 1
    encrypt_batch(drv, arena, desc, n, status, grouped=grouped)     # build valid ESP records (untimed)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0, "record generation failed"
    out = None if args.inplace else torch.empty_like(arena)
    pristine = arena.clone() if args.inplace else None
    rec_bytes = int(d["len"].astype(np.int64).sum())
    pkt_bytes = int(sizes.astype(np.int64).sum())
    ct_bytes = rec_bytes - HDR_TRAILER[cfg["alg"]] * n
    algo_bytes = rec_bytes + 16 * n + ct_bytes + n       # record + desc + PT + status

    stream = torch.cuda.Stream(device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step():
        if pristine is not None:
            arena.copy_(pristine)
        decrypt_batch(drv, arena, desc, n, status, out=out, grouped=grouped, stream=stream)

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0, "decrypt/verify failed"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.cuda.stream(stream):
        ev0.record(stream)
        for _ in range(args.steps):
            step()
        ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    ev_ms = ev0.elapsed_time(ev1)
    dt, all_pkt_bytes = aggregate(dist, world, dt, pkt_bytes, dev)
    ms_per_step = dt * 1e3 / args.steps
    value = all_pkt_bytes * args.steps / dt / 1e9
    kern_ms = ev_ms / args.steps
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9

    result = {
        "metric": "GB/s device-resident ESP AES-128-GCM decrypt, 1M×1500B pkts, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "packets_per_gpu": n, "packet_bytes": pkt_bytes // n,
                   "esp_record_bytes": rec_bytes // n, "sas_per_gpu": len(spis),
                   "sharding": "fnv1_32(spi) mod n_gpus (key_u32hash, key.c:295)",
                   "decrypt": "in-place verify-first" if args.inplace else "out-of-place single pass",
                   "value_bytes": "whole packet bytes incl. outer IPv4 header (BASELINE.json metric)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_ms": round(kern_ms, 4)},
    }
    try:
        copy = hbm_copy_gbs(arena)
        result["roofline"]["hbm_copy_gbs"] = round(copy, 1)
        result["roofline"]["frac_of_copy"] = round(achieved / copy, 4)
    except Exception as e:                       # informational only
        log("hbm copy measurement skipped: %s" % e)
    if world > 1:
        result["config"]["packets_per_rank"] = per_rank(dist, world, rank, n, dev)
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            result["roofline"]["traffic"] = json.load(f).get("hbm_bytes_per_launch")

    if not args.no_e2e:
        result["e2e_pcie"] = e2e_leg(drv, pristine if args.inplace else arena, desc, d, n, pkt_bytes,
                                     args, world, dist)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(pristine if args.inplace else arena, d, sids, keys, args,
                                              n, cfg)
    if rank == 0:
        print(json.dumps(result), flush=True)
    drv.close()
    if world > 1:
        dist.destroy_process_group()


def e2e_leg(drv, arena, desc, d, n, pkt_bytes, args, world, dist):
    """PCIe-inclusive rate (reported beside `value`, never as it): the same
    records start and end in pinned host memory; espgpu_decrypt_host streams
    them through HBM in chunks with H2D / kernels / D2H on three HIP streams."""
    import torch
    from espgpu.batch import decrypt_host
    src = arena.cpu().pin_memory()          # ciphertext records (see caller)
    h_desc = torch.from_numpy(d.view(np.uint8).copy()).pin_memory()
    h_out = torch.empty_like(src).pin_memory()
    h_st = torch.zeros(n, dtype=torch.uint8).pin_memory()
    decrypt_host(drv, src, h_desc, n, h_st, h_out, chunk=args.e2e_chunk)     # warm (allocs)
    reps = 3
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        decrypt_host(drv, src, h_desc, n, h_st, h_out, chunk=args.e2e_chunk)
    dt = time.perf_counter() - t0
    dt, all_bytes = aggregate(dist, world, dt, pkt_bytes, arena.device)
    ok = int((h_st != 0).sum()) == 0
    return {"value": round(all_bytes * reps / dt / 1e9, 2), "unit": "GB/s",
            "ms_per_batch": round(dt * 1e3 / reps, 3), "chunk_records": args.e2e_chunk,
            "status_ok": ok,
            "path": "pinned host -> H2D || kernels || D2H (3 HIP streams) -> pinned host"}


def cpu_baseline(arena, d, sids, keys, args, n, cfg):
    """The oracle (cryptosoft-shaped C restatement) on this host's cores, on a
    bounded sample of the same ciphertext records the GPU just decrypted."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:
        ncores = os.cpu_count() or 1
    threads = args.cpu_threads or max(1, min(16, ncores))
    per_thread = 32768
    m = min(n, per_thread * threads)
    if cfg["alg"] == "gcm":
        sas = [O.SA(O.CSP_MODE_AEAD, k[:-4], k[-4:]) for k in keys]
    else:
        sas = [O.SA(O.CSP_MODE_ETA, k[0], akey=k[1], mlen=12) for k in keys]
    sample = d[:m].copy()
    lo = int(sample["off4"][0]) * 4
    hi = int(sample["off4"][-1]) * 4 + int(sample["len"][-1])
    host = arena[lo:hi + 16].cpu().numpy().copy()
    sample["off4"] -= lo // 4
    sa_idx = np.searchsorted(np.array(sids), sample["sa"])
    t1, st1 = O.batch(sas, host.copy(), sample["off4"][:per_thread], sample["len"][:per_thread],
                      sa_idx[:per_thread], nthreads=1)
    tN, stN = O.batch(sas, host.copy(), sample["off4"], sample["len"], sa_idx, nthreads=threads)
    assert (st1 == 0).all() and (stN == 0).all(), "oracle rejected GPU-encrypted records"
    pkt_bytes = (sample["len"].astype(np.int64) + 20)
    return {"value": round(float(pkt_bytes.sum()) / tN / 1e9, 4), "unit": "GB/s", "cores": threads,
            "kind": "port",
            "sample": "%d %s records (%d per thread, one private session per thread), "
                      "oracle/espref.c %s restatement; 1-core rate %.4f GB/s"
                      % (m, args.config, per_thread, "swcr_gcm" if cfg["alg"] == "gcm" else "swcr_eta",
                         float(pkt_bytes[:per_thread].sum()) / t1 / 1e9)}


if __name__ == "__main__":
    main()
