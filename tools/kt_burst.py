"""Per-kernel median duration and gaps from a rocprofv3 kernel-trace database
(tools/burst_bench runs): python3 tools/kt_burst.py gpurun_out/kt/run_results.db"""
import collections
import sqlite3
import statistics as st
import sys

c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
rows = c.execute("select * from kernels order by start").fetchall()
i_n = cols.index("name") if "name" in cols else cols.index("kernel_name")
i_s, i_e = cols.index("start"), cols.index("end")
dur = collections.defaultdict(list)
for r in rows:
    dur[r[i_n][:70]].append((r[i_e] - r[i_s]) / 1e3)
for k, v in dur.items():
    print("%-70s n=%-6d med %.1f us" % (k, len(v), st.median(v)))
