#!/bin/bash
# feature-distance variants: PK_FD_DIRECT 1 (2-column waves, register double buffer), 2 (single
# buffer), 0 (LDS ring); PK_FD_PREP_VAR=1 (prep without input loads); parity tests on the default
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_configs_gpu.py tests/test_corr_pose_gpu.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
PK_FD_DIRECT=2 timeout -k 10 200 python3 tools/fd_bench.py 20 > $O/fd_bench_d2.txt 2>&1 || exit $?
for v in 1 2 0; do
  PK_FD_DIRECT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt$v -o run -- python3 tools/fd_bench.py 20 > $O/kt$v.log 2>&1 || exit $?
done
PK_FD_PREP_VAR=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/ktp -o run -- python3 tools/fd_bench.py 20 32x1024 fp32 > $O/ktp.log 2>&1
