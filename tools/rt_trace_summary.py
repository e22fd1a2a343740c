"""Merge rocprofv3 kernel and HIP API traces of an overlapped training bench: for three timed steps
from the middle of the run, the host's graph launches / event records / waits next to the first and last kernel
of every graph replay on each queue (times in us from the first of those steps' start = the end of
the clip + RMSprop launch before it).   python tools/rt_trace_summary.py <trace dir>"""
import csv
import glob
import os
import re
import sys

d = sys.argv[1]
kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
af = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
ks = sorted(csv.DictReader(open(kf[0])), key=lambda r: int(r["Start_Timestamp"]))
api = sorted(csv.DictReader(open(af[0])), key=lambda r: int(r["Start_Timestamp"])) if af else []
marks = [r for r in ks if "clip_rmsprop_kernel" in r["Kernel_Name"]]
m = len(marks) // 2  # three steps from the middle of the run (inside the timed loop)
lo, hi = int(marks[m - 2]["End_Timestamp"]), int(marks[m + 1]["End_Timestamp"])
ev = []
for a in api:
    s = int(a["Start_Timestamp"])
    if lo - 3_000_000 <= s <= hi and a["Function"] in ("hipGraphLaunch", "hipStreamWaitEvent", "hipEventRecord",
                                                       "hipLaunchKernel", "hipMemcpyWithStream"):
        ev.append((s, int(a["End_Timestamp"]), "host", a["Function"]))
prev = {}
for r in ks:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if lo <= s <= hi:
        q = "Q" + r.get("Queue_Id", "?")
        n = re.split(r"[(<]", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))[0][-40:]
        g = s - prev.get(q, s)
        if g > 8000 or "clip_rmsprop" in n or "bq_pairs" in n or "fd_top1_prep" in n or "cgt_partial" in n:
            ev.append((s, e, q, f"{n}  (gap before {g / 1e3:.1f})"))
        prev[q] = e
ev.sort()
for s, e, kind, n in ev:
    print(f"{(s - lo) / 1e3:9.1f} .. {(e - lo) / 1e3:9.1f}  {kind:5s} {n}")
