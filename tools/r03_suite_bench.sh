# Full -m gpu suite, then the default bench line and the training stream alone.
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03e} bash tools/gpu_suite_then.sh || exit $?
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG:-r03e}_bench.json 2> gpurun_out/${TAG:-r03e}_bench.err || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline-probe --train-only > gpurun_out/${TAG:-r03e}_trainonly.json 2>> gpurun_out/${TAG:-r03e}_bench.err || exit $?
for f in bench trainonly; do python -c "import json;d=json.loads(open('gpurun_out/${TAG:-r03e}_$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel'] if d.get('roofline') else None, d['roofline']['frac'] if d.get('roofline') else None)"; done
