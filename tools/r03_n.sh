export TMPDIR=/tmp
T=${TAG:-r03n}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/lin_var.py > gpurun_out/$T/lin_var.txt 2>&1 || { cat gpurun_out/$T/lin_var.txt; exit 1; }
cat gpurun_out/$T/lin_var.txt
timeout -k 10 700 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_crops_gpu.py tests/test_fps_ballquery_gpu.py tests/test_ragged_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
for nt in 1024 256; do
  PK_FPS_NT=$nt timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline-probe > gpurun_out/$T/bench_fps$nt.json 2> gpurun_out/$T/bench_fps$nt.err || exit $?
  python3 -c "import json;d=json.loads(open('gpurun_out/$T/bench_fps$nt.json').read().strip().splitlines()[-1]);print('fps_nt $nt', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_train -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > gpurun_out/$T/prof_train.json 2> gpurun_out/$T/prof_train.err || exit $?
python3 tools/kstats.py gpurun_out/$T/prof_train/run_kernel_stats.csv 28 > gpurun_out/$T/kstats.txt; head -24 gpurun_out/$T/kstats.txt
