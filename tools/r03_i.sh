# Full -m gpu suite, the default bench line and its kernel-trace stats.
export TMPDIR=/tmp
T=${TAG:-r03i}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -4 gpurun_out/$T/tests.log
case $rc in 0) ;; *) tail -60 gpurun_out/$T/tests.log; exit $rc;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$T/prof -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --steps 20 > gpurun_out/$T/prof.json 2> gpurun_out/$T/prof.err || exit $?
cat gpurun_out/$T/bench.json
timeout -k 10 200 python -u tools/rigid_bench.py 1024 2048 > gpurun_out/$T/rigid.txt 2>&1 || { cat gpurun_out/$T/rigid.txt; exit 1; }
cat gpurun_out/$T/rigid.txt
