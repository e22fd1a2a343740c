#!/bin/bash
# round-4 batch 6: weight gradients with thin operands on the pipeline; per-shape timing, new vs old.
export TMPDIR=/tmp
O=gpurun_out/r04b6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "wgrad or graphed_train" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/wg_bench.py 20 --each > $O/wg.txt 2>&1 || { tail $O/wg.txt; exit 1; }
PK_DEV=1 PK_WG_GLDS=0 timeout -k 10 200 python3 -u tools/wg_bench.py 20 --each > $O/wg_old.txt 2>&1 || { tail $O/wg_old.txt; exit 1; }
grep wgrad -A12 $O/wg.txt; grep wgrad -A12 $O/wg_old.txt
