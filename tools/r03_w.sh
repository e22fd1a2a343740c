#!/bin/bash
# feature-distance main pass limiter study: PK_FD_DIRECT 1 normal, 2 no selection, 3 no MFMA, 0 LDS ring
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
for v in 1 2 3 0; do
  PK_FD_DIRECT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt$v -o run -- python3 tools/fd_bench.py 20 32x1024 fp32 > $O/kt$v.log 2>&1 || exit $?
done
