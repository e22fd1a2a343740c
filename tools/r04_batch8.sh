#!/bin/bash
# round-4 batch 8: the ragged / TEASER tail of the suite after the thin-operand bound fix, the
# weight-gradient tests, smoke, and the weight-gradient timing (blocks capped at the CU count).
export TMPDIR=/tmp
O=gpurun_out/r04b8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ragged_gpu.py tests/test_teaser_gpu.py tests/test_model_gpu.py tests/test_pipeline_gpu.py \
  -x -v --timeout 200 --timeout-method thread -k "ragged or real or teaser or wgrad or graphed or pipelined" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 200 python3 -u tools/wg_bench.py 20 > $O/wg.txt 2>&1 || { tail $O/wg.txt; exit 1; }
grep wgrad $O/wg.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wgkt -o run -- python3 -u tools/wg_bench.py 5 > $O/wgkt.log 2>&1 || exit 1
find $O/wgkt -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | grep -i wgrad
