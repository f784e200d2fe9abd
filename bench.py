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
    "cfg1": dict(workload="cfg1: 1M x 1500B ESP AES-128-GCM decrypt, single SA", packets=1 << 20,
                 pkt=1500, skip=20, klen=16, nsa=1, mixed=False),
    "cfg2": dict(workload="cfg2: 1M x {64,256,1500,9000}B mixed-MTU ESP AES-128-GCM decrypt, 1K SAs",
                 packets=1 << 20, pkt=None, skip=20, klen=16, nsa=1024, mixed=True),
}


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
    from espgpu.esp import GCM, SecAssoc
    from espgpu.opencrypto import GpuCryptoDriver
    from espgpu.shard import spis_for_rank

    cfg = CONFIGS[args.config]
    n = cfg["packets"]
    drv = GpuCryptoDriver(device=local, max_sessions=max(16, cfg["nsa"] + 8))
    rng = np.random.default_rng(0xE5B00001 + rank)
    spis = spis_for_rank(rank, world, cfg["nsa"])
    sids, salts, keys = [], [], []
    for spi in spis:
        key = rng.integers(0, 256, cfg["klen"] + 4, dtype=np.uint8).tobytes()
        keys.append(key)
        rc, sid = drv.newsession(SecAssoc(spi, GCM, key).csp())
        assert rc == 0, drv.last_error()
        sids.append(sid)
        salts.append(int.from_bytes(key[-4:], "little"))

    # ---- synthetic records, laid out as packet slots (outer IPv4 header at 0) ----
    if cfg["mixed"]:
        sizes = rng.choice(np.array([64, 256, 1500, 9000]), n)
        sa_of = rng.integers(0, cfg["nsa"], n)
    else:
        sizes = np.full(n, cfg["pkt"])
        sa_of = np.zeros(n, dtype=np.int64)
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
    grouped = cfg["nsa"] == 1
    encrypt_batch(drv, arena, desc, n, status, grouped=grouped)     # build valid ESP records (untimed)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0, "record generation failed"
    out = None if args.inplace else torch.empty_like(arena)
    pristine = arena.clone() if args.inplace else None
    rec_bytes = int(d["len"].astype(np.int64).sum())
    pkt_bytes = int(sizes.astype(np.int64).sum())
    ct_bytes = rec_bytes - 32 * n
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
    if world > 1:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    ms_per_step = dt * 1e3 / args.steps
    value = world * pkt_bytes * args.steps / dt / 1e9
    kern_ms = ev_ms / args.steps
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9

    result = {
        "metric": "GB/s device-resident ESP AES-128-GCM decrypt, 1M×1500B pkts, 1/2/4/8 GPU",
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "packets_per_gpu": n, "packet_bytes": pkt_bytes // n,
                   "esp_record_bytes": rec_bytes // n, "sas_per_gpu": cfg["nsa"],
                   "sharding": "fnv1_32(spi) mod n_gpus (key_u32hash, key.c:295)",
                   "decrypt": "in-place verify-first" if args.inplace else "out-of-place single pass",
                   "value_bytes": "1500 B per packet (BASELINE.json metric)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_ms": round(kern_ms, 4)},
    }
    pmc = os.path.join(ROOT, "profiles", "pmc_%s.json" % args.config)
    if os.path.exists(pmc):
        with open(pmc) as f:
            result["roofline"]["traffic"] = json.load(f).get("hbm_bytes_per_launch")

    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(arena, d, sids, keys, args, n)
    if rank == 0:
        print(json.dumps(result), flush=True)
    drv.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(arena, d, sids, keys, args, n):
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
    sas = [O.SA(O.CSP_MODE_AEAD, k[:-4], k[-4:]) for k in keys]
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
            "sample": "%d cfg1 records (%d per thread, one private session per thread), "
                      "oracle/espref.c swcr_gcm restatement; 1-core rate %.4f GB/s"
                      % (m, per_thread, float(pkt_bytes[:per_thread].sum()) / t1 / 1e9)}


if __name__ == "__main__":
    main()
