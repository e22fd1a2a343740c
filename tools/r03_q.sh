# Full -m gpu suite, the default bench line (with the CPU baseline), its kernel-trace stats, and
# the inference / ragged / ransac_ref lines.
export TMPDIR=/tmp
T=${TAG:-r03q}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; tail -4 gpurun_out/$T/tests.log
case $rc in 0) ;; *) tail -60 gpurun_out/$T/tests.log; exit $rc;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit $?
cat gpurun_out/$T/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --steps 20 > gpurun_out/$T/prof.json 2> gpurun_out/$T/prof.err || exit $?
timeout -k 10 300 python -u bench.py --mode infer > gpurun_out/$T/infer.json 2> gpurun_out/$T/infer.err || exit $?
timeout -k 10 300 python -u bench.py --ragged --no-cpu-baseline > gpurun_out/$T/ragged.json 2> gpurun_out/$T/ragged.err || exit $?
for f in bench infer ragged; do python3 -c "import json;d=json.loads(open('gpurun_out/$T/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"; done
