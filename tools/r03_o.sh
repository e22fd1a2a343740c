export TMPDIR=/tmp
T=${TAG:-r03o}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_corr_pose_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python -u tools/torch_prof.py $T > gpurun_out/$T/tprof.log 2>&1 || { tail -20 gpurun_out/$T/tprof.log; exit 1; }
head -60 gpurun_out/$T/torch_prof_stacks.txt
TAG=$T/fdpmc timeout -k 10 500 bash tools/fd_pmc.sh > gpurun_out/$T/fdpmc.log 2>&1 || { tail -20 gpurun_out/$T/fdpmc.log; exit 1; }
tail -9 gpurun_out/$T/fdpmc.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (v['avg_ms'], v['ms_per_step']) for k, v in list(d['kernels'].items())[:10]})"
