#!/bin/bash
# Round-3 closing validation: full -m gpu suite, then bench lines (train default with CPU
# baseline, infer) and the kernel-trace stats of the training step.
export TMPDIR=/tmp
T=r03fin
mkdir -p gpurun_out/$T
TAG=$T bash tools/gpu_suite_then.sh || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer > gpurun_out/$T/infer.json 2> gpurun_out/$T/infer.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_step -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --steps 30 > gpurun_out/$T/prof_step.json 2> gpurun_out/$T/prof_step.err || exit $?
timeout -k 10 300 python -u bench.py --ragged --no-cpu-baseline > gpurun_out/$T/ragged.json 2> gpurun_out/$T/ragged.err || exit $?
for f in bench infer prof_step ragged; do python -c "import json;d=json.loads(open('gpurun_out/$T/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('kernel'), (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))"; done
