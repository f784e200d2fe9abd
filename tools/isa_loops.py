#!/usr/bin/env python3
"""Instruction mix of the innermost loops of one kernel in a hipcc -S listing.

  tools/isa_loops.py <file.s> <kernel-name-substring>

A loop is every basic block LLVM annotates with "in Loop: Header=BBx_y" (or
"Parent Loop BBx_y") plus the header block itself.  Per loop, prints the
counts of VALU, ds_read_b32/b128, SALU, scratch and s_waitcnt instructions
(rarely taken branches inside the loop are included)."""
import re
import sys
from collections import Counter, defaultdict


def main():
    path, kname = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^[_A-Za-z]\S*:", l) and kname in l)
    end = next(i for i in range(start, len(lines)) if "codeLenInByte" in lines[i])
    blocks, cur, loops_of = [], None, {}
    for l in lines[start:end]:
        m = re.match(r"^\.(LBB\d+_\d+):(.*)$", l)
        if m:
            cur = [m.group(1), []]
            blocks.append(cur)
            hdr = [m.group(1)] if "Loop Header" in m.group(2) else []
            loops_of[m.group(1)] = hdr
            continue
        if cur is None:
            continue
        mm = re.findall(r"(?:Header=|Parent Loop )(BB\d+_\d+)", l)
        if mm and l.strip().startswith(";"):
            loops_of[cur[0]] += ["L" + x for x in mm]
            continue
        if "Loop Header" in l and l.strip().startswith(";"):
            loops_of[cur[0]].append(cur[0])
            continue
        cur[1].append(l)
    members = defaultdict(list)
    for name, body in blocks:
        for h in set(loops_of.get(name, [])):
            members[h.lstrip("L")].append(body)
    for h, bodies in sorted(members.items(), key=lambda kv: int(kv[0].split("_")[1])):
        ins = [x.strip().split()[0] for b in bodies for x in b if x.strip() and not x.strip().startswith((";", "."))]
        c = Counter(ins)
        valu = sum(v for k, v in c.items() if k.startswith("v_"))
        salu = sum(v for k, v in c.items() if k.startswith("s_"))
        print("%-10s blocks %3d: valu %4d ds_b32 %4d ds_b128 %3d salu %4d scratch %2d waitcnt %3d" % (
            h, len(bodies), valu, c["ds_read_b32"], c["ds_read_b128"], salu,
            sum(v for k, v in c.items() if k.startswith("scratch_")), c["s_waitcnt"]))


if __name__ == "__main__":
    main()
