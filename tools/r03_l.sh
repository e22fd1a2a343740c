export TMPDIR=/tmp
T=${TAG:-r03l}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u -m pytest tests/test_ragged_gpu.py -m gpu -x -q -k "cgt" --timeout 120 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
timeout -k 10 300 python -u tools/lin_probe.py > gpurun_out/$T/lin_probe.txt 2>&1 || { cat gpurun_out/$T/lin_probe.txt; exit 1; }
cat gpurun_out/$T/lin_probe.txt
