# Counter evidence for the feature-distance kernels (pk_feat_dist_topk): configs[1] fp32 (32 x 1024^2)
# and configs[4] fp32 / bf16 (1 x 4096^2): MFMA busy vs SQ busy / VALU / LDS per launch.
export TMPDIR=/tmp
set -e
OUT=gpurun_out/${TAG:-fdpmc}
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for cfg in 32x1024:fp32 1x4096:fp32 1x4096:bf16; do
  shape=${cfg%%:*}; prec=${cfg##*:}
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/$shape$prec -o run -- python3 tools/fd_bench.py 3 $shape $prec > $OUT/$shape$prec.log 2>&1
  for kn in fd_prep_kernel fd_main_kernel fd_merge_kernel; do python3 tools/pmc_pick.py $OUT/$shape$prec $kn "$shape/$prec/$kn" >> $OUT/summary.txt; done
done
cat $OUT/summary.txt
