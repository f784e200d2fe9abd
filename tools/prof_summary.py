#!/usr/bin/env python3
"""Summarise a tools/profile.sh run into profiles/<tag>.json (+ pmc_<cfg>.json).

  python tools/prof_summary.py gpurun_out/prof_<tag> <tag> [cfg] [--out-of-place]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read (16 B/lane loads), so it is doubled; WRITE_SIZE is exact for
16-B/lane stores.  FETCH_SIZE is TCC_EA0_RDREQ x 64 B for any request size,
and quad-coalesced 64-byte groups (the ETA kernels' hash and CBC passes) make
64-B requests, so for those the doubled figure is an upper bound and the raw
one (hbm_read_bytes_raw_per_launch) a lower bound
(profiles/r6_fetch_calibration.txt).

`pipes` prices the kernel against its compute resources from the same counters
(per launch; kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs):
  lds_frac  = SQ_LDS_IDX_ACTIVE / 256 CUs / kernel cycles   (LDS-array busy share)
  valu_frac = SQ_INSTS_VALU x 2 cycles / 1024 SIMDs / kernel cycles (a wave64 VALU
              instruction holds its SIMD 2 cycles on gfx950, MI355X_MICROARCH.md:54)
and the floor each resource alone would set at that clock.  GRBM_GUI_ACTIVE
counts the whole counter window, not only the kernel, so for short launches it
implies a clock above the chip's 2.4 GHz: `pipes` is omitted (with the reason)
for kernels under 0.1 ms or whenever the implied clock exceeds 2.4 GHz.
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAX_CLOCK_GHZ = 2.4          # MI355X peak engine clock (MI355X_MICROARCH.md)


def kernel_stats(d):
    out = {}
    p = os.path.join(d, "trace", "run_kernel_stats.csv")
    for r in csv.DictReader(open(p)):
        out[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                          "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"]),
                          "pct": float(r["Percentage"])}
    return out


def steady_durations(d, name, skip):
    """Per-launch durations (ns) of kernel `name` from the kernel trace, in
    dispatch order, without the first `skip` launches (the bench's untimed
    warm-up launches, which include first-touch page mapping)."""
    p = os.path.join(d, "trace", "run_kernel_trace.csv")
    rows = [r for r in csv.DictReader(open(p)) if r["Kernel_Name"] == name]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    return [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows][skip:]


def counters(d, sub, match):
    p = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(p):
        return {}
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(p)):
        if match in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def pipes(c, kern_ms):
    """Busy shares of the LDS array and the VALU issue slots (module docstring)."""
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    ghz = cyc / (kern_ms * 1e6)
    if kern_ms < 0.1 or ghz > MAX_CLOCK_GHZ:
        return {"omitted": "kernel %.4f ms, implied clock %.2f GHz: the counter window is not the kernel"
                           % (kern_ms, ghz)}
    out = {"kernel_cycles": round(cyc), "clock_ghz": round(ghz, 3)}
    if "SQ_LDS_IDX_ACTIVE" in c:
        lds = c["SQ_LDS_IDX_ACTIVE"] / 256
        out.update(lds_cycles_per_cu=round(lds), lds_frac=round(lds / cyc, 3),
                   lds_floor_ms=round(lds / ghz / 1e6, 4))
    if "SQ_INSTS_VALU" in c:
        valu = c["SQ_INSTS_VALU"] * 2 / 1024
        out.update(valu_cycles_per_simd=round(valu), valu_frac=round(valu / cyc, 3),
                   valu_floor_ms=round(valu / ghz / 1e6, 4))
    return out


def main():
    argv = [a for a in sys.argv[1:] if a not in ("--inplace", "--out-of-place")]
    inplace = "--out-of-place" not in sys.argv      # bench.py's headline is the in-place decrypt
    d, tag = argv[0], argv[1]
    cfg = argv[2] if len(argv) > 2 else "cfg1"
    ks = kernel_stats(d)
    # the product kernel that takes the most time (the in-place bench's copies
    # of the ciphertext, one per timed step, are runtime copy kernels: never it)
    own = [k for k in ks if not k.startswith("__amd_rocclr") and "elementwise" not in k and "copy" not in k.lower()]
    dominant = max(own or ks, key=lambda k: ks[k]["pct"])
    key = dominant
    c = {}
    for sub in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_sq3"):
        c.update(counters(d, sub, key))
    steady = steady_durations(d, dominant, 10)     # profile.sh runs bench.py --warmup 10
    steady_ms = sum(steady) / len(steady) / 1e6 if steady else None
    res = {"tag": tag, "config": cfg, "dominant_kernel": dominant, "kernels": ks, "counters": c,
           "steady_avg_kernel_ms": steady_ms, "steady_launches": len(steady)}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd = 2 * c["FETCH_SIZE"] * 1024
        wr = c["WRITE_SIZE"] * 1024
        res["hbm_read_bytes_per_launch"] = rd
        res["hbm_write_bytes_per_launch"] = wr
        res["hbm_bytes_per_launch"] = rd + wr
        # FETCH_SIZE x 1: the lower bound (64-B requests, the quad-coalesced
        # reads of the ETA kernels: profiles/r6_fetch_calibration.txt)
        res["hbm_read_bytes_raw_per_launch"] = c["FETCH_SIZE"] * 1024
    if "GRBM_GUI_ACTIVE" in c:
        res["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / ks[dominant]["avg_ns"]
        res["pipes"] = pipes(c, steady_ms or ks[dominant]["avg_ns"] / 1e6)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "%s.json" % tag), "w") as f:
        json.dump(res, f, indent=1)
    if "hbm_bytes_per_launch" in res:
        # what bench.py reads: traffic is used only when dominant_kernel is the
        # kernel the bench launches
        with open(os.path.join(ROOT, "profiles", "pmc_%s%s.json" % (cfg, "_inplace" if inplace else "")),
                  "w") as f:
            json.dump({"source": "profiles/%s.json" % tag, "dominant_kernel": dominant,
                       "avg_kernel_ms": round(steady_ms or ks[dominant]["avg_ns"] / 1e6, 4),
                       "avg_kernel_ms_all_calls": round(ks[dominant]["avg_ns"] / 1e6, 4),
                       "calls": ks[dominant]["calls"],
                       "hbm_bytes_per_launch": round(res["hbm_bytes_per_launch"]),
                       "hbm_read_bytes_per_launch": round(res["hbm_read_bytes_per_launch"]),
                       "hbm_read_bytes_raw_per_launch": round(res["hbm_read_bytes_raw_per_launch"]),
                       "hbm_write_bytes_per_launch": round(res["hbm_write_bytes_per_launch"]),
                       "pipes": res.get("pipes")}, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}, indent=1))
    print("dominant:", dominant, ks[dominant])


if __name__ == "__main__":
    main()
