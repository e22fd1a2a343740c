# attention fwd+bwd at the training shape: kernel trace + one SQ counter pass (tools/attn_pmc.py)
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05attnpmc}
mkdir -p $O
timeout -k 10 60 python3 tools/attn_pmc.py 20 > $O/timing.txt 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 tools/attn_pmc.py 10 > $O/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/sq -o run -- python3 tools/attn_pmc.py 10 > $O/sq.log 2>&1
for kn in attn_fwd attn_bwd_kernel attn_bwd_dq_reduce; do python3 tools/pmc_pick.py $O/sq $kn "$kn/sq" >> $O/summary.txt; done
cat $O/timing.txt $O/summary.txt
grep -E "attn" $O/trace/run_kernel_stats.csv | cut -d, -f1-8
