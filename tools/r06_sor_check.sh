#!/bin/bash
# SOR kNN (LDS-staged pixel region): crop-formation parity tests, then the overlapped bench and
# the crop-formation kernel trace.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06sor}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_crops_gpu.py tests/test_ragged_gpu.py tests/test_formats_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/b_$rep.log 2>&1 || exit 1
  grep "^{\"metric\"" $O/b_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench rep=$rep', d['value'], d['ms_per_step'])"
done
bash tools/gpu_run.sh ${TAG:-r06sor} steptrace > /dev/null 2>&1; head -12 $O/step_window_summary.txt; grep sor_ $O/step_window_summary.txt | head -5
