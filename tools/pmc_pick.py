"""Average each counter of a rocprofv3 --pmc run over the dispatches of one kernel."""
import csv, glob, sys, collections
d, name, tag = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ""
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
acc, n = collections.defaultdict(float), collections.Counter()
for r in csv.DictReader(open(f[0])):
    if name in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
print(tag, {k: f"{acc[k] / max(n[k], 1):.4g}" for k in sorted(acc)}, flush=True)
