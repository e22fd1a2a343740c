# Pipeline/model parity, then kernel-trace stats of the graphed training step and the
# ransac_ref / ragged bench lines.
export TMPDIR=/tmp
T=${TAG:-r03f}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipeline_gpu.py tests/test_model_gpu.py > gpurun_out/$T/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline-probe > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof_train -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > gpurun_out/$T/prof_train.json 2> gpurun_out/$T/prof_train.err || exit $?
timeout -k 10 300 python -u bench.py --mode ransac_ref > gpurun_out/$T/ransac_ref.json 2> gpurun_out/$T/ransac_ref.err || exit $?
timeout -k 10 300 python -u bench.py --ragged > gpurun_out/$T/ragged.json 2> gpurun_out/$T/ragged.err || exit $?
tail -2 gpurun_out/$T/tests.log
for f in bench prof_train ransac_ref ragged; do python -c "import json;d=json.loads(open('gpurun_out/$T/$f.json').read().strip().splitlines()[-1]);print('$f', d['metric'], d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"; done
