# PMC passes over the per-point layer shapes (tools/lin_pmc.py): SQ occupancy / MFMA busy /
# stall buckets in one pass, FETCH_SIZE and WRITE_SIZE in passes of their own.
export TMPDIR=/tmp
set -e
OUT=gpurun_out/linpmc
mkdir -p $OUT
for c in rows128_64 rows64_64_mask cf32_32 cf64_64; do
  timeout -k 10 60 python tools/lin_pmc.py $c 20 >> $OUT/timing.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/$c/sq -o run -- python tools/lin_pmc.py $c 10 > $OUT/$c.sq.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$c/fetch -o run -- python tools/lin_pmc.py $c 10 > $OUT/$c.fetch.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$c/write -o run -- python tools/lin_pmc.py $c 10 > $OUT/$c.write.log 2>&1
done
for c in rows128_64 rows64_64_mask cf32_32 cf64_64; do
  for p in sq fetch write; do python tools/pmc_pick.py $OUT/$c/$p linear_ "$c/$p" >> $OUT/summary.txt; done
done
cat $OUT/timing.txt $OUT/summary.txt
