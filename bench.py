#!/usr/bin/env python3
"""Benchmark: device-resident ESP AES-128-GCM decrypt, 1M x 1500-B packets per GPU.

One step = one pass of the hot path (verify + decrypt) over one batch of
1,048,576 ESP records already resident in HBM (BASELINE.json configs[1]),
decrypted in place with verify-first semantics as F-Stack's opencrypto
consumer asks (esp_input: CRYPTO_BUF_MBUF in place, cryptosoft.c:595-633);
step k works on its own copy of the ciphertext, so no restore copy is timed.
--out-of-place times the single-pass out-of-place decrypt instead.
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
GUIDE_COPY_GBS = 6290.0        # the guide's measured float4 copy, 79 % of peak (MI355X_MICROARCH.md:36)
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


def agree_min(dist, world, value, device):
    """The smallest of the ranks' values (every rank gets it): the in-place
    copy count, so all ranks run the same timed segments."""
    if world == 1:
        return value
    import torch
    t = torch.tensor([int(value)], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


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


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv):
    """`--gpus N` without a torch.distributed launcher around us: start N ranks
    as ONE child process (`python -m torch.distributed.run --nproc-per-node N
    bench.py ...`, rendezvous on 127.0.0.1), relay rank 0's JSON line after
    checking it reports N GPUs, and return the child's exit code.  Called
    before anything touches the GPU (torch.cuda.device_count() does not
    initialise HIP on this image); the parent never execs."""
    import subprocess
    n = args.gpus
    if not args.dry_plan and os.environ.get("BENCH_SHARE_DEVICE") != "1":
        import torch
        have = torch.cuda.device_count()
        if have < n:
            log("bench.py: --gpus %d but this node has %d GPU(s); refusing to report a smaller run" % (n, have))
            return 3
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.abspath(__file__)] + argv
    log("bench.py: launching %d ranks: %s" % (n, " ".join(cmd)))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    line = None
    for raw in proc.stdout:                 # ranks' stdout; only rank 0 prints the JSON line
        s = raw.strip()
        if s.startswith("{") and '"metric"' in s:
            line = s
        else:
            sys.stderr.write(raw)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        log("bench.py: the %d-rank run exited with %d" % (n, rc))
        return rc
    if line is None:
        log("bench.py: the %d-rank run printed no result line" % n)
        return 4
    res = json.loads(line)
    if res.get("n_gpus") != n or res.get("config", {}).get("world") != n:
        log("bench.py: asked for %d GPUs, the run reports n_gpus=%s world=%s"
            % (n, res.get("n_gpus"), res.get("config", {}).get("world")))
        return 5
    print(line, flush=True)
    return 0


def dry_plan(args, world, rank, local):
    """--dry-plan: the rank logic of a run without a GPU (gloo, CPU tensors):
    each rank plans its share of the config's packets (SPI-hash sharding) and
    rank 0 prints the JSON line's shape with world, packets_per_rank and the
    device ids, so the N-rank launch path is testable on a CPU host."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    cfg = dict(CONFIGS[args.config])
    if args.packets:
        cfg["packets"] = args.packets
    rng = np.random.default_rng(0xE5B00001 + rank)
    spis, sa_of, sizes = plan_packets(cfg, rank, world, rng)
    cpu = torch.device("cpu")
    n = len(sizes)
    res = {"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world, "steps": 0,
           "warmup": 0, "dry_plan": True,
           "config": {"workload": cfg["workload"], "world": world,
                      "packets_per_rank": per_rank(dist, world, rank, n, cpu),
                      "sas_per_rank": per_rank(dist, world, rank, len(spis), cpu),
                      "device_per_rank": per_rank(dist, world, rank, local, cpu)}}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


METRIC = "GB/s device-resident ESP AES-128-GCM decrypt, 1M×1500B pkts, 1/2/4/8 GPU"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="cfg1", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="0 = every core of this process's CPU share (affinity and cgroup quota)")
    ap.add_argument("--cpu-runs", type=int, default=5, help="cpu_baseline: median of this many runs")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out-of-place", action="store_true",
                    help="time the out-of-place single-pass decrypt as the headline (default: the "
                         "verify-first in-place decrypt, the opencrypto contract, with the out-of-place "
                         "rate reported beside it)")
    ap.add_argument("--inplace", action="store_true", help="the default headline mode (kept for old scripts)")
    ap.add_argument("--no-inplace-leg", action="store_true",
                    help="skip the side measurement of the other decrypt mode")
    ap.add_argument("--no-encrypt-leg", action="store_true", help="skip the encrypt-direction side measurement")
    ap.add_argument("--no-packed-leg", action="store_true",
                    help="skip the packed-output side measurement (espgpu_decrypt_batch_packed)")
    ap.add_argument("--tuning", action="append", default=[],
                    help="experiment: espgpu_set_tuning key=value (e.g. grid=300; gcm_opts and eta_opts need the knobs build)")
    ap.add_argument("--nsa", type=int, default=0,
                    help="experiment: override the config's SA count (0 = the config's own)")
    ap.add_argument("--no-e2e", action="store_true", help="skip the PCIe-inclusive host-to-host leg")
    ap.add_argument("--e2e-chunk", type=int, default=65536, help="records per pipelined step")
    ap.add_argument("--out-pad", type=int, default=0,
                    help="experiment: extra bytes per record in the out-of-place buffer (layout probes)")
    ap.add_argument("--sizes", default="",
                    help="experiment: comma list of packet sizes drawn uniformly instead of the config's")
    ap.add_argument("--sa-runs", action="store_true",
                    help="experiment: lay each SA's records out back to back (placement probe)")
    ap.add_argument("--sa-even", action="store_true",
                    help="experiment: the same SAs and placement rule, but every SA gets the same record count")
    ap.add_argument("--planner", action="store_true",
                    help="experiment: run single-SA batches through the device planner too (not grouped)")
    ap.add_argument("--dry-plan", action="store_true",
                    help="test aid: run the N-rank launch and each rank's packet plan on gloo/CPU, no GPU")
    ap.add_argument("--packets", type=int, default=0, help="with --dry-plan: packets per GPU override")
    argv = sys.argv[1:]
    args = ap.parse_args(argv)
    inplace = not args.out_of_place
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        log("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, args.gpus))
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_plan:
        dry_plan(args, world, rank, local)
        return

    import torch
    import torch.distributed as dist
    # rehearsal of the N-rank path on a one-GPU box (never a measurement):
    # BENCH_SHARE_DEVICE=1 puts every rank on device 0 and BENCH_DIST_BACKEND=gloo
    # replaces RCCL, which refuses two ranks on one device
    if os.environ.get("BENCH_SHARE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    else:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from espgpu.batch import decrypt_batch, encrypt_batch
    from espgpu.esp import CBC_SHA1, GCM, SecAssoc
    from espgpu.opencrypto import GpuCryptoDriver

    cfg = dict(CONFIGS[args.config])
    if args.nsa:
        cfg["nsa"] = args.nsa
        cfg["workload"] += " [SA count overridden: %d]" % args.nsa
    rng = np.random.default_rng(0xE5B00001 + rank)
    spis, sa_of, sizes = plan_packets(cfg, rank, world, rng)
    if args.sizes:
        sizes = np.random.default_rng(0xE5B0000F + rank).choice(
            np.array([int(x) for x in args.sizes.split(",")]), len(sizes))
        cfg["workload"] += " [packet sizes overridden: %s]" % args.sizes
    if args.sa_even:
        nsa_here = len(spis)
        sa_of = np.random.default_rng(0xE5B00010 + rank).permutation(np.arange(len(sa_of)) % nsa_here)
        cfg["workload"] += " [equal record count per SA]"
    if args.sa_runs:
        order = np.argsort(sa_of, kind="stable")
        sa_of, sizes = sa_of[order], sizes[order]
        cfg["workload"] += " [records grouped by SA]"
    n = len(sizes)
    drv = GpuCryptoDriver(device=local, max_sessions=max(16, len(spis) + 8))
    for kv in args.tuning:
        k, _, v = kv.partition("=")
        assert drv.lib.espgpu_set_tuning(drv.ctx, k.encode(), int(v)) == 0, "tuning %s refused" % kv
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
    grouped = len(spis) == 1 and not args.planner
    if args.planner:
        cfg["workload"] += " [device planner]"
    encrypt_batch(drv, arena, desc, n, status, grouped=grouped)     # build valid ESP records (untimed)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0, "record generation failed"
    out = None if inplace else torch.empty(total + args.out_pad * n, dtype=torch.uint8, device=dev)
    # In place, every timed step needs ciphertext: step k decrypts its own copy
    # of the records (`arena` itself stays ciphertext for the side legs), as
    # many copies as K steps when HBM holds them (288 GB: 20 x 1.5 GB), else
    # timed segments of as many steps with the copies restored between them,
    # outside the timed region.  Each copy is cold (1.5 GB >> L2 + MALL).
    if inplace:
        free = torch.cuda.mem_get_info(dev)[0]
        ncopy = max(1, min(args.steps, int(free * 0.6) // total))
        ncopy = agree_min(dist, world, ncopy, dev)   # the same segments on every rank
        bufs = [arena.clone() for _ in range(ncopy)]
    else:
        bufs = [arena]
    rec_bytes = int(d["len"].astype(np.int64).sum())
    pkt_bytes = int(sizes.astype(np.int64).sum())
    ct_bytes = rec_bytes - HDR_TRAILER[cfg["alg"]] * n
    algo_bytes = rec_bytes + 16 * n + ct_bytes + n       # record + desc + PT + status

    stream = torch.cuda.Stream(device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def step(k):
        decrypt_batch(drv, bufs[k % len(bufs)], desc, n, status, out=out, grouped=grouped, stream=stream)

    def restore():
        if inplace:
            with torch.cuda.stream(stream):
                for b in bufs:
                    b.copy_(arena)
        torch.cuda.synchronize()

    with torch.cuda.stream(stream):
        for k in range(args.warmup):
            if inplace:
                bufs[0].copy_(arena)
            step(0)
        if inplace:
            bufs[0].copy_(arena)
    torch.cuda.synchronize()
    knobs = any(kv.split("=")[0] in ("gcm_opts", "eta_opts") and not kv.endswith("=0") for kv in args.tuning)
    assert knobs or int((status != 0).sum()) == 0, "decrypt/verify failed"   # knobs break results on purpose
    dt, ev_ms, done = 0.0, 0.0, 0
    while done < args.steps:
        seg = min(len(bufs), args.steps - done)
        if done:
            restore()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            ev0.record(stream)
            for k in range(seg):
                step(k)
            ev1.record(stream)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt += time.perf_counter() - t0
        ev_ms += ev0.elapsed_time(ev1)
        done += seg
    assert knobs or int((status != 0).sum()) == 0, "decrypt/verify failed in the timed steps"
    del bufs
    dt, all_pkt_bytes = aggregate(dist, world, dt, pkt_bytes, dev)
    ms_per_step = dt * 1e3 / args.steps
    value = all_pkt_bytes * args.steps / dt / 1e9
    kern_ms = ev_ms / args.steps
    achieved = algo_bytes / (kern_ms * 1e-3) / 1e9

    assert world == args.gpus, "n_gpus %d != --gpus %d" % (world, args.gpus)
    result = {
        "metric": METRIC,
        "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic",
        "config": {"workload": cfg["workload"], "packets_per_gpu": n, "packet_bytes": pkt_bytes // n,
                   "esp_record_bytes": rec_bytes // n, "sas_per_gpu": len(spis),
                   "sharding": "fnv1_32(spi) mod n_gpus (key_u32hash, key.c:295)",
                   "decrypt": ("in place, verify first (the opencrypto contract, cryptosoft.c:595-633)"
                               if inplace else "out-of-place single pass"),
                   "value_bytes": "whole packet bytes incl. outer IPv4 header (BASELINE.json metric)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": None,
                     "algorithmic_bytes_per_launch": algo_bytes,
                     "kernel_ms": round(kern_ms, 4)},
    }
    # against the guide's measured copy ceiling (a torch copy here reaches less)
    result["roofline"]["guide_copy_gbs"] = GUIDE_COPY_GBS
    result["roofline"]["frac_of_guide_copy"] = round(achieved / GUIDE_COPY_GBS, 4)
    try:
        copy = hbm_copy_gbs(arena)
        result["roofline"]["hbm_copy_gbs"] = round(copy, 1)
        result["roofline"]["frac_of_copy"] = round(achieved / copy, 4)
    except Exception as e:                       # informational only
        log("hbm copy measurement skipped: %s" % e)
    result["config"]["world"] = world
    result["config"]["packets_per_rank"] = per_rank(dist, world, rank, n, dev)
    result["config"]["device_per_rank"] = per_rank(dist, world, rank, local, dev)
    if world > 1:
        result["config"]["distinct_devices"] = len(set(result["config"]["device_per_rank"]))
    if inplace:
        result["config"]["inplace_copies"] = ncopy
    kernel = launched_kernel(cfg, inplace)
    result["roofline"]["kernel"] = kernel
    result["roofline"].update(profile_traffic(args.config, inplace, kernel, kern_ms))
    if not args.no_inplace_leg:
        leg = side_leg(drv, arena, desc, n, status, grouped, stream, pkt_bytes,
                       algo_bytes, world, dist, launched_kernel(cfg, not inplace), not inplace)
        result["inplace" if not inplace else "out_of_place"] = leg

    if not args.no_packed_leg and cfg["alg"] == "gcm":
        result["packed_out"] = packed_leg(drv, arena, desc, d, n, status, grouped, stream, pkt_bytes,
                                          algo_bytes, world, dist)

    if not args.no_encrypt_leg:
        result["encrypt"] = encrypt_leg(drv, arena, desc, n, status, grouped, stream, pkt_bytes, world, dist, cfg)

    if not args.no_e2e:
        result["e2e_pcie"] = e2e_leg(drv, arena, desc, d, n, pkt_bytes,
                                     args, world, dist)
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(arena, d, sids, keys, args,
                                              n, cfg)
        try:
            result["cpu_openssl"] = cpu_openssl(arena, d, sids, keys, args,
                                                n, cfg)
        except Exception as e:                   # informational only (needs tools/libossl_esp.so)
            log("cpu_openssl skipped: %s" % e)
    if rank == 0:
        print(json.dumps(result), flush=True)
    drv.close()
    if world > 1:
        dist.destroy_process_group()


def launched_kernel(cfg, inplace):
    """Source name of the kernel the timed loop launches (the one the roofline
    prices): gcm_kernel<MODE, 1024, S, STAGE> with MODE 3 = decrypt in place,
    verify first, in one pass (a failed record's keystream XORed back over it;
    MODE 2, the two-pass in-place decrypt, is built with GCM_INPLACE_ONEPASS=0
    only), MODE 0 = out of place, S = 4 lanes per record (every bench
    config has >= 32K records: the small-batch S = 8 kernel is not launched),
    STAGE false (device-resident records);
    eta_kernel<3, 768, -2> (out of place) / <2, 1024, -2> (in place) for CBC +
    HMAC-SHA1 (verify pass, then the block-parallel decrypt of the verified
    records; -2 = the launch for SHA-1 / SHA2-256 sessions, esp_cbc.hip
    CK_NARROW)."""
    if cfg["alg"] == "gcm":
        return "gcm_kernel<%d, 1024, 4, false>" % (3 if inplace else 0)
    return "eta_kernel<2, 1024, -2>" if inplace else "eta_kernel<3, 768, -2>"   # verify-first two-pass


def profile_traffic(config, inplace, kernel, kern_ms):
    """HBM traffic per launch from the committed rocprofv3 summary of this
    configuration (tools/prof_summary.py), used ONLY if that summary's dominant
    kernel is the kernel this run launched; its average duration is reported
    beside the live kernel_ms so the two can be compared."""
    name = "pmc_%s%s.json" % (config, "_inplace" if inplace else "")
    path = os.path.join(ROOT, "profiles", name)
    out = {"traffic": None, "profile": None}
    if not os.path.exists(path):
        return out
    with open(path) as f:
        pm = json.load(f)
    dom = pm.get("dominant_kernel", "")
    out["profile"] = {"file": "profiles/" + name, "source": pm.get("source"), "dominant_kernel": dom,
                      "avg_kernel_ms": pm.get("avg_kernel_ms")}
    if kernel in dom:
        out["traffic"] = pm.get("hbm_bytes_per_launch")
        if pm.get("hbm_read_bytes_raw_per_launch") is not None:
            # FETCH_SIZE x 1: the reads if every request were 64 B (quad-
            # coalesced loads; traffic doubles them per the guide's rule, an
            # upper bound for those kernels: profiles/r6_fetch_calibration.txt)
            out["traffic_reads_raw"] = pm["hbm_read_bytes_raw_per_launch"]
        if pm.get("pipes"):
            # the compute resources of the same kernel: LDS-array and VALU-issue
            # busy shares and the floor each would set alone (tools/prof_summary.py)
            out["pipes"] = pm["pipes"]
        if pm.get("avg_kernel_ms"):
            out["profile"]["avg_over_live"] = round(pm["avg_kernel_ms"] / kern_ms, 3)
    else:
        out["profile"]["mismatch"] = "profile is of another kernel: traffic not used"
    return out


def side_leg(drv, arena, desc, n, status, grouped, stream, pkt_bytes, algo_bytes, world, dist, kernel,
             inplace):
    """The other decrypt mode on the same records, beside the headline: the
    verify-first in-place decrypt (d_out == d_arena: failed records keep their
    ciphertext; GCM in one pass that rolls a failed record back, ETA in two
    passes; a restore copy before every launch, untimed) or the out-of-place
    single pass.  Only the decrypt launches are timed (HIP events on the
    stream), median of 5."""
    import torch
    from espgpu.batch import decrypt_batch
    work = arena.clone() if inplace else None
    dst = None if inplace else torch.empty_like(arena)
    reps = 5
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps + 1)]
    with torch.cuda.stream(stream):
        for e0, e1 in evs:
            if inplace:
                work.copy_(arena)
            e0.record(stream)
            decrypt_batch(drv, work if inplace else arena, desc, n, status, out=dst, grouped=grouped,
                          stream=stream)
            e1.record(stream)
    torch.cuda.synchronize()
    ok = int((status != 0).sum()) == 0
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs[1:])[reps // 2]
    del work, dst
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=arena.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(pkt_bytes)], dtype=torch.float64, device=arena.device)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        ms, pkt_bytes = float(t.item()), float(b.item())
    return {"value": round(pkt_bytes / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "kernel_ms": round(ms, 4),
            "achieved_algorithmic_GBps": round(algo_bytes / (ms * 1e-3) / 1e9, 1),
            "status_ok": ok, "timing": "median of %d launches, HIP events around the decrypt only" % reps,
            "kernel": kernel + (" (verify-first, in place)" if inplace else " (out of place, single pass)")}


def packed_leg(drv, arena, desc, d, n, status, grouped, stream, pkt_bytes, algo_bytes, world, dist):
    """The same out-of-place decrypt with a packed output
    (espgpu_decrypt_batch_packed: record i's plaintext at out + i*stride,
    stride = the largest payload rounded up to 128 bytes, every output line
    written whole), beside the headline's record layout; not the headline."""
    import torch
    from espgpu.batch import decrypt_batch_packed
    ct_max = int(d["len"].max()) - HDR_TRAILER["gcm"]
    stride = (ct_max + 127) // 128 * 128
    out = torch.empty(n * stride, dtype=torch.uint8, device=arena.device)
    reps = 5
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps + 1)]
    with torch.cuda.stream(stream):
        for e0, e1 in evs:
            e0.record(stream)
            decrypt_batch_packed(drv, arena, desc, n, status, out, stride, grouped=grouped, stream=stream)
            e1.record(stream)
    torch.cuda.synchronize()
    ok = int((status != 0).sum()) == 0
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs[1:])[reps // 2]
    del out
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=arena.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(pkt_bytes)], dtype=torch.float64, device=arena.device)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        ms, pkt_bytes = float(t.item()), float(b.item())
    return {"value": round(pkt_bytes / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "kernel_ms": round(ms, 4),
            "achieved_algorithmic_GBps": round(algo_bytes / (ms * 1e-3) / 1e9, 1),
            "frac": round(algo_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "out_stride": stride,
            "status_ok": ok, "timing": "median of %d launches, HIP events around the decrypt only" % reps,
            "api": "espgpu_decrypt_batch_packed (plaintext of record i at out + i*stride; not the headline)"}


def encrypt_leg(drv, arena, desc, n, status, grouped, stream, pkt_bytes, world, dist, cfg):
    """The esp_output direction on the same records (espgpu_encrypt_batch, in
    place: payload encrypted, ICV written), beside the headline.  Encrypting
    any bytes is valid work, so the launches run back to back on a copy of the
    arena; HIP events around the encrypt launches only."""
    import torch
    from espgpu.batch import encrypt_batch
    work = arena.clone()
    reps = 5
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps + 1)]
    with torch.cuda.stream(stream):
        for e0, e1 in evs:
            e0.record(stream)
            encrypt_batch(drv, work, desc, n, status, grouped=grouped, stream=stream)
            e1.record(stream)
    torch.cuda.synchronize()
    ok = int((status != 0).sum()) == 0
    ms = sorted(e0.elapsed_time(e1) for e0, e1 in evs[1:])[reps // 2]
    del work
    if world > 1:
        t = torch.tensor([ms], dtype=torch.float64, device=arena.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        b = torch.tensor([float(pkt_bytes)], dtype=torch.float64, device=arena.device)
        dist.all_reduce(b, op=dist.ReduceOp.SUM)
        ms, pkt_bytes = float(t.item()), float(b.item())
    # (CBC + HMAC: the chain and the ICV in one pass, esp_cbc.hip launch_eta)
    kernel = "gcm_kernel<1, 1024, 4, false>" if cfg["alg"] == "gcm" else "eta_kernel<4, 1024, 2>"
    return {"value": round(pkt_bytes / (ms * 1e-3) / 1e9, 2), "unit": "GB/s", "kernel_ms": round(ms, 4),
            "status_ok": ok, "timing": "median of %d launches, HIP events around the encrypt only" % reps,
            "kernel": kernel + " (in place, ICV written)"}


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
    res = {"value": round(all_bytes * reps / dt / 1e9, 2), "unit": "GB/s",
           "ms_per_batch": round(dt * 1e3 / reps, 3), "chunk_records": args.e2e_chunk,
           "status_ok": ok,
           "path": "pinned host -> H2D || kernels || D2H (3 HIP streams) -> pinned host"}
    try:
        # the ceiling of this leg: the same bytes copied H2D and D2H at once
        # (two streams, no kernel), as GB/s of packets in each direction
        bw = pcie_bidir_gbs(src, h_out, arena)
        res["pcie_bidir_copy_gbs"] = round(bw, 2)
        res["frac_of_copy"] = round(res["value"] / bw, 3)
    except Exception as e:                        # informational only
        log("pcie copy measurement skipped: %s" % e)
    return res


def pcie_bidir_gbs(h_src, h_dst, d_buf, reps=3):
    """Bytes per second in each direction with an H2D copy of h_src into one
    half of the device and a D2H copy of the other half into h_dst running
    concurrently on two streams."""
    import torch
    nb = h_src.numel()
    d_in = torch.empty(nb, dtype=torch.uint8, device=d_buf.device)
    d_out = torch.empty(nb, dtype=torch.uint8, device=d_buf.device)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(s1):
            d_in.copy_(h_src, non_blocking=True)
        with torch.cuda.stream(s2):
            h_dst.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del d_in, d_out
    return nb * reps / dt / 1e9


def cpu_share():
    """Cores this process may use: its affinity set, capped by the cgroup CPU
    quota (the GPU box gives each job a share of a larger machine)."""
    try:
        aff = sorted(os.sched_getaffinity(0))
    except AttributeError:
        aff = list(range(os.cpu_count() or 1))
    share, src = len(aff), "sched_getaffinity"
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                q = int(quota) // int(period)
                if 0 < q < share:
                    share, src = q, "cgroup cpu.max %s/%s" % (quota, period)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0 and 0 < q // p < share:
            share, src = q // p, "cgroup cfs_quota_us"
    except (OSError, ValueError):
        pass
    return share, src, aff


def cpu_info(cpus):
    """(model name, physical cores among `cpus`) from /proc/cpuinfo."""
    model, phys, cur = None, set(), {}
    try:
        for line in open("/proc/cpuinfo"):
            if not line.strip():
                if cur.get("processor") in cpus:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "processor":
                cur["processor"] = int(v)
            elif k in ("physical id", "core id"):
                cur[k] = v
            elif k == "model name" and model is None:
                model = v
        if cur.get("processor") in cpus:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    return model, len(phys) or None


def cpu_baseline(arena, d, sids, keys, args, n, cfg):
    """The oracle (cryptosoft-shaped C restatement) on this host's cores: the
    same ciphertext records the GPU just decrypted, every core of the job's
    CPU share, median of --cpu-runs runs; plus the 1-core rate."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    share, src, aff = cpu_share()
    threads = args.cpu_threads or share
    model, phys = cpu_info(set(aff[:threads]) if len(aff) >= threads else set(aff))
    per_thread = 65536
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
    one = min(m, 16384)
    t1, st1 = O.batch(sas, host.copy(), sample["off4"][:one], sample["len"][:one], sa_idx[:one], nthreads=1)
    runs = []
    for _ in range(max(1, args.cpu_runs)):
        tN, stN = O.batch(sas, host.copy(), sample["off4"], sample["len"], sa_idx, nthreads=threads)
        assert (stN == 0).all(), "oracle rejected GPU-encrypted records"
        runs.append(tN)
    assert (st1 == 0).all(), "oracle rejected GPU-encrypted records"
    tN = sorted(runs)[len(runs) // 2]
    pkt_bytes = (sample["len"].astype(np.int64) + cfg["skip"])
    return {"value": round(float(pkt_bytes.sum()) / tN / 1e9, 4), "unit": "GB/s", "cores": threads,
            "kind": "port", "median_of": len(runs),
            "runs_s": [round(t, 3) for t in runs],
            "cpu_model": model, "cores_physical": phys, "cpu_share": share, "cpu_share_source": src,
            "one_core_GBps": round(float(pkt_bytes[:one].sum()) / t1 / 1e9, 4),
            "sample": "%d %s records (all of this rank's records up to %d per thread) on %d threads, "
                      "oracle/espref.c %s restatement, median of %d runs (%.1f CPU-seconds in all)"
                      % (m, args.config, per_thread, threads,
                         "swcr_gcm" if cfg["alg"] == "gcm" else "swcr_eta", len(runs),
                         sum(runs) * threads)}


def cpu_openssl(arena, d, sids, keys, args, n, cfg):
    """OpenSSL 3 EVP (AES-NI / VAES / PCLMULQDQ) on the same records and
    threads as cpu_baseline: NOT the reference path (F-Stack's kernel crypto
    is cryptosoft's table code), a comparison point only."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import ossl_esp
    import ssl
    if not ossl_esp.available():
        raise RuntimeError("tools/libossl_esp.so not built")
    share, _, _ = cpu_share()
    threads = args.cpu_threads or share
    m = min(n, 65536 * threads)
    sample = d[:m].copy()
    lo = int(sample["off4"][0]) * 4
    hi = int(sample["off4"][-1]) * 4 + int(sample["len"][-1])
    host = arena[lo:hi + 16].cpu().numpy().copy()
    sample["off4"] -= lo // 4
    sa_idx = np.searchsorted(np.array(sids), sample["sa"])
    if cfg["alg"] == "gcm":
        kw = dict(alg="gcm", ckeys=[k[:-4] for k in keys], salts=[k[-4:] for k in keys], mlen=16)
    else:
        kw = dict(alg="cbc_sha1", ckeys=[k[0] for k in keys], akeys=[k[1] for k in keys], mlen=12)
    # out of place (so the sample stays ciphertext), REPS times over per run,
    # so a run lasts ~1 s and the cgroup quota's 100-ms periods average out
    REPS = 8
    out = np.empty_like(host)
    runs = []
    for _ in range(max(1, args.cpu_runs)):
        t, st = ossl_esp.batch_decrypt(arena=host, off4=sample["off4"], lens=sample["len"], sa_idx=sa_idx,
                                       nthreads=threads, out=out, reps=REPS, **kw)
        assert (st == 0).all(), "OpenSSL rejected GPU-encrypted records"
        runs.append(t / REPS)
    t1, st1 = ossl_esp.batch_decrypt(arena=host, off4=sample["off4"][:16384], lens=sample["len"][:16384],
                                     sa_idx=sa_idx[:16384], nthreads=1, out=out, reps=REPS, **kw)
    assert (st1 == 0).all()
    t1 /= REPS
    tN = sorted(runs)[len(runs) // 2]
    pkt_bytes = (sample["len"].astype(np.int64) + cfg["skip"])
    return {"value": round(float(pkt_bytes.sum()) / tN / 1e9, 3), "unit": "GB/s", "cores": threads,
            "kind": "openssl, not the reference path", "library": ssl.OPENSSL_VERSION,
            "median_of": len(runs), "runs_s": [round(t, 4) for t in runs],
            "one_core_GBps": round(float(pkt_bytes[:16384].sum()) / t1 / 1e9, 3),
            "sample": "the cpu_baseline records (%d) on %d threads, EVP %s out of place, verify + decrypt, "
                      "%d passes per run (seconds per pass)"
                      % (m, threads, "AES-GCM" if cfg["alg"] == "gcm" else "AES-CBC + HMAC-SHA1", REPS)}


if __name__ == "__main__":
    main()
