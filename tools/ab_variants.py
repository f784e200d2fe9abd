#!/usr/bin/env python3
"""A/B the GCM kernel variants in ONE process, interleaved rounds (cfg1 shape).
  python tools/ab_variants.py [--variants 0,1,2,3] [--rounds 5] [--steps 10] [--grid 0]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "f-stack_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--pkt", type=int, default=1500)
    ap.add_argument("--no-check", action="store_true", help="for measurement-only variants")
    args = ap.parse_args()
    import torch
    from espgpu.batch import decrypt_batch, encrypt_batch
    from espgpu.esp import GCM, SecAssoc
    from espgpu.opencrypto import GpuCryptoDriver
    drv = GpuCryptoDriver()
    key = bytes(range(20))
    rc, sid = drv.newsession(SecAssoc(0x1234, GCM, key).csp())
    n, pkt = args.n, args.pkt
    d = np.zeros(n, dtype=[("off4", "<u4"), ("len", "<u2"), ("sa", "<u2"), ("esn_hi", "<u4"), ("salt", "<u4")])
    d["off4"] = (np.arange(n, dtype=np.int64) * pkt + 20) // 4
    d["len"] = pkt - 20
    d["sa"] = sid
    d["salt"] = int.from_bytes(key[-4:], "little")
    desc = torch.from_numpy(d.view(np.uint8).copy()).cuda()
    arena = torch.randint(0, 256, (n * pkt + 64,), dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.uint8, device="cuda")
    encrypt_batch(drv, arena, desc, n, st, grouped=True)
    out = torch.empty_like(arena)
    variants = [int(v) for v in args.variants.split(",")]
    grids = [int(g) for g in args.grids.split(",")]
    res = {(v, g): [] for v in variants for g in grids}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(args.rounds):
        for v in variants:
            for g in grids:
                drv.lib.espgpu_set_tuning(drv.ctx, b"gcm_variant", v)
                drv.lib.espgpu_set_tuning(drv.ctx, b"grid", g)
                decrypt_batch(drv, arena, desc, n, st, out=out, grouped=True)
                torch.cuda.synchronize()
                assert args.no_check or int((st != 0).sum()) == 0, (v, g)
                e0.record()
                for _ in range(args.steps):
                    decrypt_batch(drv, arena, desc, n, st, out=out, grouped=True)
                e1.record()
                torch.cuda.synchronize()
                res[(v, g)].append(e0.elapsed_time(e1) / args.steps)
    for (v, g), t in res.items():
        t = np.array(t)
        print("variant %d grid %4d: median %.4f ms  min %.4f  -> %.1f GB/s" %
              (v, g, np.median(t), t.min(), n * pkt / np.median(t) / 1e6))


if __name__ == "__main__":
    main()
