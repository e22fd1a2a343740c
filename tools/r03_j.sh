# Overlap-head / rigidity parity after the latency fixes, rigidity timing + kernel trace + PMC,
# per-point-layer limiter study, and a quick headline line.
export TMPDIR=/tmp
T=${TAG:-r03j}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py -m gpu -x -q -k "overlap or rigid or fused" --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 200 python -u tools/rigid_bench.py 1024 2048 > gpurun_out/$T/rigid.txt 2>&1 || { cat gpurun_out/$T/rigid.txt; exit 1; }
cat gpurun_out/$T/rigid.txt
RIGID_ITERS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/rtrace -o run -- python3 tools/rigid_bench.py 1024 > gpurun_out/$T/rtrace.log 2>&1 || exit $?
TAG=$T/rpmc timeout -k 10 500 bash tools/rigid_pmc.sh > gpurun_out/$T/rpmc.log 2>&1 || { tail -20 gpurun_out/$T/rpmc.log; exit 1; }
cat gpurun_out/$T/rpmc.log | tail -12
timeout -k 10 200 python -u tools/lin_var.py > gpurun_out/$T/lin_var.txt 2>&1 || { cat gpurun_out/$T/lin_var.txt; exit 1; }
cat gpurun_out/$T/lin_var.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: v['avg_ms'] for k, v in d['kernels'].items() if 'overlap' in k or 'linear' in k})"
