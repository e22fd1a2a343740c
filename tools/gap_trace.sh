# kernel trace of the overlapped step, then the training stream's gaps (tools/gap_trace.py)
export TMPDIR=/tmp
out=gpurun_out/${TAG:-gaps}
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 $1 > $out/bench.log 2>&1 || exit 1
python3 tools/gap_trace.py $(find $out/tr -name "*kernel_trace.csv" | head -1) $out/bench.log 5 > $out/gaps.txt 2>&1
find $out/tr -type f -delete
cat $out/gaps.txt
