#!/usr/bin/env python3
"""Per-kernel resource usage from hipcc's -Rpass-analysis=kernel-resource-usage
remarks: VGPRs, AGPRs, SGPRs, spills, LDS, occupancy (measurement aid).

  hipcc ... -c f.hip -Rpass-analysis=kernel-resource-usage 2> f.res
  python3 tools/kres.py f.res [filter]
"""
import re
import subprocess
import sys

FIELDS = [("VGPRs", "vgpr"), ("AGPRs", "agpr"), ("SGPRs", "sgpr"), ("VGPRs Spill", "vspill"),
          ("SGPRs Spill", "sspill"), ("LDS Size [bytes/block]", "lds"), ("Occupancy [waves/SIMD]", "occ")]


def parse(path):
    out, cur = {}, None
    for ln in open(path):
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        if cur is None:
            continue
        for key, short in FIELDS:
            m = re.search(r"\s" + re.escape(key) + r": (\d+)", ln)
            if m:
                out[cur][short] = int(m.group(1))
    return out


def demangle(names):
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
        return r.stdout.splitlines()
    except OSError:
        return names


def main():
    res = parse(sys.argv[1])
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    names = list(res)
    for n, d in zip(names, demangle(names)):
        if flt not in d:
            continue
        r = res[n]
        short = re.sub(r"espgpu::\(anonymous namespace\)::", "", d)
        print("%-60s vgpr %3s sgpr %3s vspill %3s sspill %3s lds %6s occ %s" % (
            short[:60], r.get("vgpr"), r.get("sgpr"), r.get("vspill"), r.get("sspill"), r.get("lds"), r.get("occ")))


if __name__ == "__main__":
    main()
