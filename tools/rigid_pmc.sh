# Counter evidence for the inference critical path's VALU kernels: pk_rigidity_filter (round-3
# packed path and round 2's gather path, configs[1]: 32 crops x 5120 candidates) and pk_ransac
# (the reference's 4 x 10^6 hypotheses x 760 correspondences). One SQ pass, FETCH / WRITE passes.
export TMPDIR=/tmp
set -e
OUT=gpurun_out/${TAG:-rigidpmc}
mkdir -p $OUT
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
export RIGID_ITERS=3
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/rsq -o run -- python3 tools/rigid_bench.py 1024 > $OUT/rsq.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/rfetch -o run -- python3 tools/rigid_bench.py 1024 > $OUT/rfetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $OUT/qsq -o run -- python3 bench.py --mode ransac_ref --steps 2 --warmup 1 --eager --no-cpu-baseline --no-roofline-probe > $OUT/qsq.log 2>&1
for kn in rigid_gather_kernel rigid_pair2_kernel rigid_pair_kernel rigid_reduce_kernel rigid_compact_kernel rigid_compact_pts_kernel; do
  python3 tools/pmc_pick.py $OUT/rsq $kn "$kn/sq" >> $OUT/summary.txt
  python3 tools/pmc_pick.py $OUT/rfetch $kn "$kn/fetch" >> $OUT/summary.txt
done
for kn in ransac_fit_kernel ransac_score_kernel ransac_reduce_kernel; do python3 tools/pmc_pick.py $OUT/qsq $kn "$kn/sq" >> $OUT/summary.txt; done
cat $OUT/summary.txt
