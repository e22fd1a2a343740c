#!/bin/bash
# GPU-box runner: each step under its own timeout; stop at the first failure or runtime
# fault (HSA exception text in the step's log), so nothing else touches a faulted GPU.
#   tools/gpu_run.sh <tag> <steps...>   steps: tests | smoke | bench | prof | pmc | kbench
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
fault() { grep -q "HSA_STATUS_ERROR\|hipErrorLaunchFailure\|Memory access fault" "$1"; }
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" >&2
  timeout -k 10 "$to" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$out/status.txt"
  if fault "$out/$name.log"; then echo "$name: GPU FAULT" >> "$out/status.txt"; tail -30 "$out/$name.log"; exit 3; fi
  if [ $rc -ne 0 ]; then tail -40 "$out/$name.log"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    icp) run icp 200 python bench.py --mode icp ;;
    teaser) run teaser 200 python bench.py --mode teaser --steps 5 --warmup 1 ;;
    ops) run ops 300 python bench.py --mode operators --batch 8 --steps 3 --warmup 1 ;;
    infer) run infer 300 python bench.py --mode infer ;;
    corr) run corr 300 python bench.py --mode corr4096 ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    testsall) run testsall 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    benchq) run benchq 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ;;
    benche) run benche 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-probe --eager ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline-probe
          find "$out/prof" -type f ! -name "*stats.csv" -delete ;;
    kbench) run kbench 300 python tools/kbench.py ;;
    steptrace) run steptrace_bench 400 rocprofv3 --kernel-trace --output-format csv -d "$out/steptrace" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0
               grep "^{\"metric\"" "$out/steptrace_bench.log" | tail -1 > "$out/steptrace.json"
               python tools/step_window_summary.py $(find "$out/steptrace" -name "*kernel_trace.csv" | head -1) "$out/steptrace.json" > "$out/step_window_summary.txt" 2>&1
               find "$out/steptrace" -type f -delete ;;
    steptrace_pc1) DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 run steptrace_pc1_bench 400 rocprofv3 --kernel-trace --output-format csv -d "$out/steptrace_pc1" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0
               grep "^{\"metric\"" "$out/steptrace_pc1_bench.log" | tail -1 > "$out/steptrace_pc1.json"
               python tools/step_window_summary.py $(find "$out/steptrace_pc1" -name "*kernel_trace.csv" | head -1) "$out/steptrace_pc1.json" > "$out/step_window_summary_pc1.txt" 2>&1
               find "$out/steptrace_pc1" -type f -delete ;;
    steptrace_to) run steptrace_to_bench 400 rocprofv3 --kernel-trace --output-format csv -d "$out/steptrace_to" -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0 --train-only
               grep "^{\"metric\"" "$out/steptrace_to_bench.log" | tail -1 > "$out/steptrace_to.json"
               python tools/step_window_summary.py $(find "$out/steptrace_to" -name "*kernel_trace.csv" | head -1) "$out/steptrace_to.json" > "$out/step_window_summary_train_only.txt" 2>&1
               find "$out/steptrace_to" -type f -delete ;;
    fdstamps) PK_FD_VAR=13 run fdstamps 200 python tools/fd_stamps.py ;;
    mvprobe) run mvprobe 200 python tools/mfma_valu_probe.py ;;
    moprobe) run moprobe 200 python tools/mfma_order_probe.py ;;
    pmcstep) TAG=$tag/pmcstep run pmcstep 700 bash tools/pmc_step.sh ;;
    kprof) run kprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kprof" -o run -- python tools/kbench.py
          find "$out/kprof" -type f ! -name "*stats.csv" -delete ;;
    pmcm) run pmcm 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$out/pmcm" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager --probe-steps 1
          python tools/mfma_util.py "$out/pmcm" fd_main_kernel attn_fwd attn_bwd wgrad_grouped_kernel linear_fwd_rows linear_fwd_cf nce_pass > "$out/mfma_util_step.json" 2>&1
          find "$out/pmcm" -type f -name "*.csv" -size +2M -delete ;;
    pmc) run pmcf 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out/pmcf" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager --probe-steps 1
         run pmcw 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out/pmcw" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --eager --probe-steps 1
         python tools/pmc_summary.py "$out/pmcf" "$out/pmcw" "$out/pmc_traffic.json" > "$out/pmc_summary.log" 2>&1
         find "$out/pmcf" "$out/pmcw" -type f -name "*.csv" -size +2M -delete ;;
    fdb) run fdb 300 python tools/fd_bench.py ;;
    fdpmc) run fdpmc1 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$out/fdpmc1" -o run -- python tools/fd_bench.py 5 32x1024 fp32 1,5
           python tools/mfma_util.py "$out/fdpmc1" fd_top1_kernel fd_top1_prep_kernel fd_top1_merge fd_main_direct_kernel fd_prep_kernel fd_merge_kernel > "$out/mfma_util.json" 2>&1
           python tools/pmc_pick.py "$out/fdpmc1" fd_ > "$out/fd_pmc_counters.txt" 2>&1 || true ;;
    tprof) run tprof 300 python tools/torch_prof.py "$tag" ;;
    mprobe) run mprobe 300 python tools/memset_graph_probe.py ;;
    mprobe_nopc) DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run mprobe_nopc 300 python tools/memset_graph_probe.py ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
cat "$out/status.txt"
