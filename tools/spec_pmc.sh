# Spectral diffusion per-kernel HBM traffic (FETCH_SIZE, then WRITE_SIZE: separate passes) and
# timing at the training step's shape (64 crops x 1024 points: both shapes of a configs[1] batch)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-specpmc}
mkdir -p $OUT
timeout -k 10 120 python3 -u tools/spec_bench.py 64 1024 > $OUT/bench.txt 2>&1 || exit 1
cat $OUT/bench.txt
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o run -- python3 tools/spec_bench.py 64 1024 > $OUT/$c.log 2>&1 || exit 1
  for k in spec_reduce_mfma_kernel spec_combine4_kernel spec_expand_mfma_kernel; do
    python3 tools/pmc_pick.py $OUT/$c $k "$c $k" >> $OUT/summary.txt || exit 1
  done
done
cat $OUT/summary.txt
