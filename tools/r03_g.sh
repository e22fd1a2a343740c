# Model parity (ragged channels-first layers), attention PMC passes, ragged bench, step kernel stats.
export TMPDIR=/tmp
T=${TAG:-r03g}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_ragged_gpu.py > gpurun_out/$T/tests.log 2>&1 || { tail -30 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
bash tools/attn_pmc.sh > gpurun_out/$T/attn_pmc.txt 2>&1 || { cat gpurun_out/$T/attn_pmc.txt; exit 1; }
cat gpurun_out/$T/attn_pmc.txt
timeout -k 10 300 python -u bench.py --ragged --no-cpu-baseline > gpurun_out/$T/ragged.json 2> gpurun_out/$T/ragged.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_train -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > gpurun_out/$T/prof_train.json 2> gpurun_out/$T/prof_train.err || exit $?
for f in ragged prof_train; do python -c "import json;d=json.loads(open('gpurun_out/$T/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'])"; done
