#!/bin/bash
# after the feature-distance rework: parity tests, fd_bench, train / infer / infer-2048 / corr4096 bench lines
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_corr_pose_gpu.py tests/test_ragged_gpu.py tests/test_pipeline_gpu.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
timeout -k 10 200 python3 tools/fd_bench.py 20 > $O/fd_bench.txt 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_train.json 2> $O/bench_train.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer --no-cpu-baseline > $O/bench_infer.json 2> $O/bench_infer.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer --points 2048 --no-cpu-baseline > $O/bench_infer2048.json 2> $O/bench_infer2048.err || exit $?
timeout -k 10 300 python -u bench.py --mode corr4096 --no-cpu-baseline > $O/bench_corr4096.json 2> $O/bench_corr4096.err || exit $?
for f in train infer infer2048 corr4096; do python -c "import json;d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['unit'], d['ms_per_step'], d.get('roofline',{}).get('kernel'), d.get('roofline',{}).get('frac'))"; done
