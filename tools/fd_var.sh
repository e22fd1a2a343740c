#!/bin/bash
# Feature-distance A/B (dev library): PK_FD_PATH (0 default, 1 rows + cols, 2 two-pass, 3 fused
# 8-wave) and, for the default top-1 pass, PK_FD_VAR limiter variants (1 no selection, 2 no
# MFMAs, 3 neither, 4 compiler schedule, 5 value-only selection, 6 integer select, 7 AGPR
# accumulators, 8 med3 + compare + select, 9 value-only med3); fp32,
# graph-replayed (tools/fd_bench.py).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fdvar}
mkdir -p $OUT
SHAPE=${SHAPE:-32x1024}
for v in ${VARS:-0 1 2 3 4 5 6 7 8 9}; do
  PK_DEV=1 PK_FD_VAR=$v timeout -k 10 120 python3 -u tools/fd_bench.py 20 $SHAPE fp32 2>&1 | grep feat_dist | sed "s/^/var=$v /" >> $OUT/var.txt || exit 1
done
cat $OUT/var.txt
