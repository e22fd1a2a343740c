#!/bin/bash
# feature-distance: LDS-ring vs direct main pass, parity tests on the default (direct)
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_corr_pose_gpu.py -m gpu > $O/tests.txt 2>&1 &&
PK_FD_DIRECT=1 timeout -k 10 200 python3 tools/fd_bench.py 20 > $O/fd_bench_direct.txt 2>&1 &&
PK_FD_DIRECT=0 timeout -k 10 200 python3 tools/fd_bench.py 20 32x1024 fp32 > $O/fd_bench_ring.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run -- python3 tools/fd_bench.py 20 32x1024 fp32 > $O/kt.log 2>&1
rc=$?
tail -3 $O/tests.txt; cat $O/fd_bench_direct.txt $O/fd_bench_ring.txt
exit $rc
