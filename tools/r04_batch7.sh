#!/bin/bash
# round-4 batch 7: scalar-base glds issue (weight gradients + per-point layers): tests, per-shape
# weight-gradient timing, layer A/B, census of one training step.
export TMPDIR=/tmp
O=gpurun_out/r04b7
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "wgrad or graphed_train or linear or encoder or dpfmnet or relu or block or overlap or attn_prop" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/wg_bench.py 20 --each > $O/wg.txt 2>&1 || { tail $O/wg.txt; exit 1; }
grep wgrad -A12 $O/wg.txt
TAG=r04b7/lin bash tools/lin_ab.sh || exit 1
timeout -k 10 200 python3 -u tools/lin_census.py > $O/census.txt 2>&1 || { tail $O/census.txt; exit 1; }
head -3 $O/census.txt; grep "pk_linear_wgrad_grouped" $O/census.txt
