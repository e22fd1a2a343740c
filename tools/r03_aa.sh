#!/bin/bash
# pk_copy_rows for the attention node's concatenation + the ragged feature-distance edge test
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_capi.py -m gpu > $O/tests.txt 2>&1 || { tail -40 $O/tests.txt; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > $O/prof.json 2> $O/prof.err || exit $?
tail -2 $O/tests.txt
python -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
