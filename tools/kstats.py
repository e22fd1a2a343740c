"""Per-kernel summary of a rocprofv3 --stats CSV: python tools/kstats.py <run_kernel_stats.csv> [per]
(per = calls of one step's once-per-step kernel family, to print per-step time)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)
    return n[:70]


tot = sum(float(r["TotalDurationNs"]) for r in rows if "spin_kernel" not in r["Name"])
print(f"total {tot / 1e6:.2f} ms ({tot / 1e3 / per:.1f} us per step at per={per:g})")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if "spin_kernel" in r["Name"]:
        continue
    t = float(r["TotalDurationNs"])
    if t < 0.003 * tot:
        break
    print(f"{short(r['Name']):70s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:8.2f} us {t / 1e3 / per:8.1f} us/step")
