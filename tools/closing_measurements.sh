#!/bin/bash
# Closing measurements of a round: the headline train bench (with CPU baseline), inference at
# configs[1] and at the configs[3] shard, (f1) operators, the step kernel trace, and the PMC
# traffic passes (SKIP_OPS / SKIP_PMC: leave those two out). Each step under its own limit; the first
# failure ends the script.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-close}
mkdir -p $O
step() { local name=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err || { echo "$name failed"; tail -20 $O/$name.err; exit 1; }; tail -c 400 $O/$name.out; echo; }
step train 600 python3 -u bench.py
step infer 300 python3 -u bench.py --mode infer
step infer2048 300 python3 -u bench.py --mode infer --points 2048 --no-cpu-baseline
step ragged 600 python3 -u bench.py --ragged --no-cpu-baseline
[ -n "$SKIP_OPS" ] || step ops 400 python3 -u bench.py --mode operators --batch 8 --steps 3 --warmup 1
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-probe
find $O/prof -type f ! -name "*stats.csv" -delete
# the timed steps alone (no eager warm-up / probe steps in the window): tools/step_window_summary.py
step steptrace 400 rocprofv3 --kernel-trace --output-format csv -d $O/steptrace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0
python3 tools/step_window_summary.py $(find $O/steptrace -name "*kernel_trace.csv" | head -1) $O/steptrace.out > $O/step_window_summary.txt || exit 1
find $O/steptrace -type f -delete
head -30 $O/step_window_summary.txt
[ -n "$SKIP_PMC" ] && exit 0
TAG=${TAG:-close}/pmc bash tools/pmc_step.sh > $O/pmc.out 2>&1 || { tail -20 $O/pmc.out; exit 1; }
tail -5 $O/pmc.out
