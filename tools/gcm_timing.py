#!/usr/bin/env python3
"""Kernel-time A/B harness for the GCM decrypt kernel (measurement only).

  python tools/gcm_timing.py [--records N] [--rec-len L] [--reps R] [--opts K ...]

Times espgpu_decrypt_batch (out of place, grouped, one AES-128-GCM SA) over N
random records of L bytes with HIP events on the launch stream, once per
measurement-knob setting.  Records are random bytes, not valid ESP: every tag check
fails, which is the same work as a passing one (the kernel decrypts
regardless in out-of-place mode), so a variant whose arithmetic is
deliberately wrong can still be timed.  Prints one JSON line per variant."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f-stack_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--rec-len", type=int, default=1480)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--opts", type=int, nargs="*", default=[0],
                    help="measurement knobs (libespgpu built with make KNOBS=1): 1 no loads/stores, "
                         "2 no GHASH, 4 no AES rounds 3+, 8 no stores, 16 no loads, 32 no table staging, "
                         "64 no final multiply")
    ap.add_argument("--grid", type=int, default=0)
    ap.add_argument("--tuning", action="append", default=[], help="espgpu_set_tuning key=value (e.g. gcm_lanes=8)")
    args = ap.parse_args()
    import torch
    from espgpu.batch import decrypt_batch
    from espgpu.esp import GCM, SecAssoc
    from espgpu.opencrypto import GpuCryptoDriver
    drv = GpuCryptoDriver(device=0, max_sessions=16)
    rc, sid = drv.newsession(SecAssoc(0x1234, GCM, bytes(range(20))).csp())
    assert rc == 0
    n, rl = args.records, args.rec_len
    slot = (rl + 20 + 3) & ~3
    d = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")])
    d["off4"] = (np.arange(n, dtype=np.int64) * slot + 20) // 4
    d["len"] = rl
    d["sa"] = sid
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    arena = torch.randint(0, 256, (n * slot + 64,), dtype=torch.uint8, device="cuda")
    out = torch.empty_like(arena)
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    stream = torch.cuda.Stream()
    algo = n * (rl + 16) + n * (rl - 32) + n
    drv.lib.espgpu_set_tuning(drv.ctx, b"grid", args.grid)
    for kv in args.tuning:
        k, v = kv.split("=")
        assert drv.lib.espgpu_set_tuning(drv.ctx, k.encode(), int(v)) == 0, kv
    for s in args.opts:
        if s:
            assert drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_opts", s) == 0, "knobs need a KNOBS=1 build"
        with torch.cuda.stream(stream):
            for _ in range(3):
                decrypt_batch(drv, arena, desc, n, st, out=out, grouped=True, stream=stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                decrypt_batch(drv, arena, desc, n, st, out=out, grouped=True, stream=stream)
            e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(json.dumps({"opts": s, "grid": args.grid, "records": n, "rec_len": rl, "kernel_ms": round(ms, 4),
                          "algo_GBps": round(algo / ms / 1e6, 1)}), flush=True)
    drv.close()


if __name__ == "__main__":
    main()
