# step kernel profile of the headline train bench (rocprofv3 --kernel-trace --stats), summarized
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05prof}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-probe > $O/bench.out 2>&1 || { tail -20 $O/bench.out; exit 1; }
find $O/prof -type f ! -name "*stats.csv" ! -name "*kernel_trace.csv" -delete
python3 tools/kstats.py $(find $O/prof -name "*kernel_stats.csv" | head -1) 12 > $O/summary.txt
head -70 $O/summary.txt
