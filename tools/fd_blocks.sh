#!/bin/bash
# Feature-distance top-1 grid-size sweep (dev library PK_FD_BLOCKS) x limiter variants (PK_FD_VAR)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fdblocks}
mkdir -p $OUT
for nb in ${BLOCKS:-256 512 1024}; do
  for v in ${VARS:-0 12}; do
    PK_DEV=1 PK_FD_BLOCKS=$nb PK_FD_VAR=$v timeout -k 10 120 python3 -u tools/fd_bench.py 20 32x1024 fp32 2>&1 | grep feat_dist | sed "s/^/blocks=$nb var=$v /" >> $OUT/var.txt || exit 1
  done
done
cat $OUT/var.txt
