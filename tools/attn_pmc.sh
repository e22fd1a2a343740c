# PMC passes over the training step's attention (tools/attn_pmc.py): SQ busy / MFMA busy /
# VALU / LDS bank conflicts in one pass, FETCH_SIZE and WRITE_SIZE in passes of their own.
export TMPDIR=/tmp
set -e
OUT=gpurun_out/attnpmc
mkdir -p $OUT
timeout -k 10 60 python tools/attn_pmc.py 20 > $OUT/timing.txt 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python tools/attn_pmc.py 10 > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o run -- python tools/attn_pmc.py 10 > $OUT/sq.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python tools/attn_pmc.py 10 > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python tools/attn_pmc.py 10 > $OUT/write.log 2>&1
for kn in attn_fwd attn_bwd_kernel attn_bwd_dq_reduce; do
  for p in sq fetch write; do python tools/pmc_pick.py $OUT/$p $kn "$kn/$p" >> $OUT/summary.txt; done
done
cat $OUT/timing.txt $OUT/summary.txt
cat $OUT/trace/run_kernel_stats.csv 2>/dev/null | head -12 || true
