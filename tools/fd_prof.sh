#!/bin/bash
# Feature-distance profile at configs[1] fp32 top-1: kernel trace (durations per kernel) and one
# SQ counter pass; summaries in gpurun_out/$TAG/.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fdprof}
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/fd_bench.py 5 32x1024 fp32 > $OUT/kt.log 2>&1 || exit 1
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
find $OUT/kt -type f ! -name "*stats.csv" -delete
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d $OUT/pmc -o run -- python3 tools/fd_bench.py 3 32x1024 fp32 > $OUT/pmc.log 2>&1 || exit 1
for kn in fd_fused_kernel fd_merge_kernel fd_prep_kernel fd_main_direct; do python3 tools/pmc_pick.py $OUT/pmc $kn "$kn" >> $OUT/summary.txt; done
find $OUT/pmc -type f -name "*.csv" -size +2M -delete
cat $OUT/summary.txt
cut -d, -f1-8 $OUT/kernel_stats.csv | head -8
