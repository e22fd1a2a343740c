#!/bin/bash
# Closing check of the final tree: full -m gpu suite, smoke(), default bench line.
export TMPDIR=/tmp
T=r03fin2
mkdir -p gpurun_out/$T
TAG=$T bash tools/gpu_suite_then.sh || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 1; }
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
tail -1 gpurun_out/$T/smoke.txt
python -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], d['pose_err']['end_to_end_max_abs_dT'])"
