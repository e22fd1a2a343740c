#!/bin/bash
# Model / pipeline / configs GPU tests, a 40-step overlapped bench and a kernel-trace profile of
# the replayed step (O=gpurun_out/$TAG). The first failing step ends the script.
O=gpurun_out/${TAG:-r05step}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py tests/test_fps_ballquery_gpu.py tests/test_crops_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline-probe --steps 40 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-probe > /dev/null 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -type f ! -name "*stats.csv" -delete
python3 - "$O/prof/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[1:40]:
    print(f"{r['Name'][:64]:66s}{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.2f} us {float(r['TotalDurationNs'])/12e3:8.1f} us/step")
PY
