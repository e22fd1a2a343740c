# SOR kNN counters (tools/sor_bench.py): one SQ pass, one TA/TCP pass
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sorpmc}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/sq -o run -- python3 tools/sor_bench.py 5 > $O/sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $O/ta -o run -- python3 tools/sor_bench.py 5 > $O/ta.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/sor_bench.py 5 > $O/tr.log 2>&1 || exit 1
for p in sq ta; do python3 tools/pmc_pick.py $O/$p sor_knn "sor_knn/$p"; done
grep -h sor_ $(find $O/tr -name "*kernel_stats.csv") | cut -d, -f1-5
