#!/bin/bash
# round-4 batch 2: weight-gradient pipeline tests + A/B (census of one training step, with and
# without PK_WG_GLDS), the rigidity filter A/B and its kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r04b2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "wgrad or graphed or pipelined or train_and_infer" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/lin_census.py > $O/census.txt 2>&1 || { tail $O/census.txt; exit 1; }
PK_DEV=1 PK_WG_GLDS=0 timeout -k 10 200 python3 -u tools/lin_census.py > $O/census_old.txt 2>&1 || { tail $O/census_old.txt; exit 1; }
grep -A30 "pk_linear_wgrad_grouped" $O/census.txt; grep "pk_linear_wgrad_grouped" $O/census_old.txt
timeout -k 10 200 python3 -u tools/rigid_bench.py 1024 2048 > $O/rigid.txt 2>&1 || { tail $O/rigid.txt; exit 1; }
cat $O/rigid.txt
RIGID_ITERS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rprof -o rp -- python3 -u tools/rigid_bench.py 2048 > $O/rigid_prof.txt 2>&1 || exit 1
find $O/rprof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-4 | head -20
