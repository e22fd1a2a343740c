#!/bin/bash
# deferred IR in PipelinedTrainer: pipeline / distributed tests, bench with PK_DEFER_IR=1 vs 0
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_pipeline_gpu.py tests/test_distributed_gpu.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
for r in 1 2; do
for v in 1 0; do
PK_DEFER_IR=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 > $O/bench_defer$v.$r.json 2> $O/bench_defer$v.$r.err || exit $?
python -c "import json;d=json.loads(open('$O/bench_defer$v.$r.json').read().strip().splitlines()[-1]);print('defer$v', d['value'], d['ms_per_step'], d['ir'], d['loss'])"
done
done
