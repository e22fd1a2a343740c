# kernel + HIP runtime API trace of the overlapped bench (no counters): when does the host
# submit each graph launch relative to the GPU timeline
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d $out/tr -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 $2 > $out/bench.log 2>&1
python tools/rt_trace_summary.py $out/tr > $out/summary.txt 2>&1
find $out/tr -type f -name "*.csv" ! -name "*kernel_trace.csv" ! -name "*hip_api_trace.csv" -delete
cat $out/summary.txt | head -80
