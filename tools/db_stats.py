"""Per-kernel summary (calls, average, total) of a rocprofv3 rocpd database (the default output
format when --output-format is not given): python tools/db_stats.py <run_results.db> [per] [out.csv]
(per = steps, to print per-step time; out.csv: the same rows in rocprofv3's kernel_stats CSV columns)."""
import csv
import re
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else cols[0])
rows = c.execute(f"select {name_col}, count(*), avg(end - start), sum(end - start) from kernels group by {name_col}").fetchall()
rows.sort(key=lambda r: -r[3])
tot = sum(r[3] for r in rows)


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)[:70]


print(f"total {tot / 1e6:.2f} ms ({tot / 1e3 / per:.1f} us per step at per={per:g})")
for n, k, a, s in rows:
    if s < 0.003 * tot:
        break
    print(f"{short(n):70s} {k:5d} {a / 1e3:8.2f} us {s / 1e3 / per:8.1f} us/step")
if len(sys.argv) > 3:
    with open(sys.argv[3], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for n, k, a, s in rows:
            w.writerow([n, k, int(s), int(a), f"{100.0 * s / tot:.4f}"])
