#!/bin/bash
# round-4 batch 5: 3-stage pipelined inference (tests + bench at 2048 points, 2 vs 3 stages), the
# compare + select feature-distance selection, and the grouped weight-gradient microbench with a
# kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r04b5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_pipeline_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "infer or feat_dist or chain" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
for st in 2 3; do
  timeout -k 10 300 python3 -u bench.py --mode infer --points 2048 --no-cpu-baseline --infer-stages $st > $O/infer2048_s$st.json 2> $O/infer2048_s$st.err || { tail $O/infer2048_s$st.err; exit 1; }
  cut -c1-330 $O/infer2048_s$st.json
done
VARS="0" TAG=r04b5/fd bash tools/fd_var.sh || exit 1
timeout -k 10 120 python3 -u tools/wg_bench.py > $O/wg.txt 2>&1 || { tail $O/wg.txt; exit 1; }
PK_DEV=1 PK_WG_GLDS=0 timeout -k 10 120 python3 -u tools/wg_bench.py > $O/wg_old.txt 2>&1 || { tail $O/wg_old.txt; exit 1; }
cat $O/wg.txt $O/wg_old.txt | grep wgrad
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wgkt -o run -- python3 -u tools/wg_bench.py 5 > $O/wgkt.log 2>&1 || exit 1
find $O/wgkt -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | head -12
