#!/usr/bin/env python3
"""Print the kernel stats of a rocprofv3 --stats CSV (name, calls, average us)."""
import csv
import sys
for path in sys.argv[1:]:
    print(path)
    for r in list(csv.DictReader(open(path)))[:10]:
        print("  %-100s %4s %10.1f us" % (r["Name"][:100], r["Calls"], float(r["AverageNs"]) / 1e3))
