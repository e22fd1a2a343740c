export TMPDIR=/tmp
O=gpurun_out/r06inftr; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python bench.py --mode infer --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/b.log 2>&1 || exit 1
f=$(find $O/tr -name "*kernel_stats.csv" | head -1)
python3 tools/kstats.py $f 12 | head -30
find $O/tr -type f ! -name "*kernel_stats.csv" -delete
