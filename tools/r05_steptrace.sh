#!/bin/bash
# Kernel trace of the timed steps alone (tools/step_window_summary.py): no eager warm-up or
# probe steps in the window, both streams counted.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05steptrace}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/bench.out 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 tools/step_window_summary.py $(find $O/tr -name "*kernel_trace.csv" | head -1) $O/bench.out > $O/step_window_summary.txt || exit 1
find $O/tr -type f -delete
head -70 $O/step_window_summary.txt
