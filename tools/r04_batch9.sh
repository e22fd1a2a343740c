#!/bin/bash
# round-4 batch 9: the ragged / TEASER tail after the rank-aware C_gt check, wgrad timing (blocks
# capped at the CU count), smoke, operators split (f1: host flips vs device).
export TMPDIR=/tmp
O=gpurun_out/r04b9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ragged_gpu.py tests/test_teaser_gpu.py tests/test_configs_gpu.py tests/test_model_gpu.py tests/test_pipeline_gpu.py \
  -v --timeout 200 --timeout-method thread -k "ragged or real or teaser or wgrad or graphed or pipelined or configs2" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; grep -q "HSA_STATUS_ERROR\|illegal memory\|Memory access fault" $O/tests.txt && exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/wgkt -o run -- python3 -u tools/wg_bench.py 5 > $O/wgkt.log 2>&1 || exit 1
find $O/wgkt -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | grep -i wgrad
find $O/wgkt -type f ! -name "*stats.csv" -delete
timeout -k 10 300 python3 -u tools/ops_split.py 8 2000 > $O/ops_split.txt 2>&1 || { tail $O/ops_split.txt; exit 1; }
tail -1 $O/ops_split.txt
exit $rc
