"""Kernel-trace timeline of the feature-distance launches (rocprofv3 --kernel-trace CSV): per
kernel name the average duration, and the average gap from one kernel's end to the next one's
start within the replayed graph.   python tools/fd_trace.py <run_kernel_trace.csv>"""
import csv
import re
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
short = lambda n: re.sub(r"\(.*", "", n.replace("void ", "").replace("(anonymous namespace)::", ""))[:60]  # noqa
dur, gap = defaultdict(list), defaultdict(list)
prev = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    k = short(r["Kernel_Name"])
    dur[k].append(e - s)
    if prev is not None and 0 <= s - prev[1] < 20000:
        gap[(prev[0], k)].append(s - prev[1])
    prev = (k, e)
for k, v in dur.items():
    print(f"{k:60s} n={len(v):4d} avg {sum(v) / len(v) / 1e3:8.2f} us")
for (a, b), v in gap.items():
    print(f"gap {a[:28]:28s} -> {b[:28]:28s} n={len(v):4d} avg {sum(v) / len(v) / 1e3:6.2f} us")
