export TMPDIR=/tmp
T=${TAG:-r03r}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "wgrad or pipeline or graphed or train_step or fused or dpfm" --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], {k: (v['avg_ms'], v['ms_per_step']) for k, v in list(d['kernels'].items())[:8]})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_train -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > gpurun_out/$T/prof_train.json 2> gpurun_out/$T/prof_train.err || exit $?
python3 tools/kstats.py gpurun_out/$T/prof_train/run_kernel_stats.csv 28 > gpurun_out/$T/kstats.txt; head -12 gpurun_out/$T/kstats.txt
