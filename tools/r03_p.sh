export TMPDIR=/tmp
T=${TAG:-r03p}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_fps_ballquery_gpu.py tests/test_crops_gpu.py tests/test_ragged_gpu.py tests/test_pipeline_gpu.py tests/test_formats_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['avg_ms'], v['ms_per_step']) for k, v in list(d['kernels'].items())[:6]})"
timeout -k 10 300 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/$T/infer.json 2> gpurun_out/$T/infer.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/infer.json').read().strip().splitlines()[-1]);print('infer', d['value'], d['ms_per_step'], {k: (v['avg_ms'], v['ms_per_step']) for k, v in list(d['kernels'].items())[:6]})"
