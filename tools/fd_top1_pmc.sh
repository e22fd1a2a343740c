# Counter evidence for the one-launch top-1 feature-distance kernel (fd_top1_kernel) at
# configs[1] (32 x 1024^2 fp32): two --pmc passes (each within the SQ block's 8 slots)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-fdt1pmc}
mkdir -p $OUT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 tools/fd_bench.py 3 32x1024 fp32 > $OUT/p$i.log 2>&1 || exit 1
  python3 tools/pmc_pick.py $OUT/p$i fd_top1_kernel "pass$i" >> $OUT/summary.txt || exit 1
done
cat $OUT/summary.txt
