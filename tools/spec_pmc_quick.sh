#!/bin/bash
# Spectral diffusion alone: timing (tools/spec_bench.py) and FETCH / WRITE passes (one counter each).
export TMPDIR=/tmp
O=gpurun_out/${TAG:-specq}; mkdir -p $O
timeout -k 10 120 python3 tools/spec_bench.py 64 1024 > $O/timing.txt 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/$c -o run -- python3 tools/spec_bench.py 64 1024 > /dev/null 2>&1 || exit 1
done
python3 - "$O" <<'PY'
import csv, glob, sys, collections, re
O = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    tot = collections.defaultdict(float); n = collections.Counter()
    for f in glob.glob(f"{O}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != c or "spec_" not in r["Kernel_Name"]:
                continue
            k = re.search(r"spec_\w+(<[^>]*>)?", r["Kernel_Name"]).group(0)
            tot[k] += float(r["Counter_Value"]); n[k] += 1
    print(c, {k: round(v / n[k] * 1024 * (2 if c == "FETCH_SIZE" else 1) / 1e6, 2) for k, v in tot.items()}, "MB per launch")
PY
tail -3 $O/timing.txt
