#!/bin/bash
# feature-distance rework check: parity tests, fd_bench, per-kernel trace
export TMPDIR=/tmp
set -o pipefail
mkdir -p gpurun_out/r03u
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_corr_pose_gpu.py -m gpu > gpurun_out/r03u/tests.txt 2>&1 &&
timeout -k 10 200 python3 tools/fd_bench.py 20 > gpurun_out/r03u/fd_bench.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r03u/kt -o run -- python3 tools/fd_bench.py 20 32x1024 fp32 > gpurun_out/r03u/kt.log 2>&1
rc=$?
tail -3 gpurun_out/r03u/tests.txt; cat gpurun_out/r03u/fd_bench.txt
exit $rc
