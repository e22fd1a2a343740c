#!/bin/bash
# HBM traffic of the training step's kernel families (MI355X_MICROARCH.md, HBM/rocprofv3): one
# counter per pass (FETCH_SIZE, then WRITE_SIZE), eager steps without warm-up so every dispatch
# belongs to a counted step, each pass under its own time limit; tools/pmc_summary.py turns the
# passes into bytes per launch (per entry-point call where the bench's probe counted the calls).
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmcstep}
mkdir -p $OUT
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- \
    python3 bench.py --steps 3 --warmup 0 --no-cpu-baseline --eager > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
done
python3 tools/pmc_summary.py $OUT/FETCH_SIZE $OUT/WRITE_SIZE $OUT/pmc_traffic.json $OUT/bench_FETCH_SIZE.json > $OUT/summary.log 2>&1 || exit 1
find $OUT/FETCH_SIZE $OUT/WRITE_SIZE -type f -name "*.csv" -size +4M -delete
cat $OUT/pmc_traffic.json | head -80
