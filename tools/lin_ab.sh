#!/bin/bash
# Per-point layer A/B: tools/lin_bench.py with the production library (LDS-DMA rows pipeline) and
# with the dev library's PK_ROWS_GLDS=0 (round 3's fragment-load rows kernel).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-linab}
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/lin_bench.py > $OUT/glds.txt 2>&1 || { tail -20 $OUT/glds.txt; exit 1; }
PK_DEV=1 PK_ROWS_GLDS=0 timeout -k 10 200 python3 -u tools/lin_bench.py > $OUT/frag.txt 2>&1 || { tail -20 $OUT/frag.txt; exit 1; }
paste -d'\n' $OUT/glds.txt $OUT/frag.txt | grep -v amdgpu.ids
