# kernel trace of graph-replayed training steps (no eager probe): per-step kernel time vs wall time
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 $2 > $out/bench.log 2>&1
python tools/step_trace_summary.py $out/tr/run_kernel_trace.csv $out/bench.log 200 > $out/summary.txt 2>&1
find $out/tr -type f -delete
head -70 $out/summary.txt
