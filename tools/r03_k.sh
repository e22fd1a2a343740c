# Bandwidth calibration (torch copy / sum by launch size), per-point layer shapes (fragment vs
# LDS-staged rows kernel), the inference line with the packed rigidity path, and the training
# step's kernel trace (CSV).
export TMPDIR=/tmp
T=${TAG:-r03k}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/bw_probe.py > gpurun_out/$T/bw_probe.txt 2>&1 || { cat gpurun_out/$T/bw_probe.txt; exit 1; }
cat gpurun_out/$T/bw_probe.txt
timeout -k 10 200 python -u tools/lin_bench.py > gpurun_out/$T/lin_bench.txt 2>&1 || { cat gpurun_out/$T/lin_bench.txt; exit 1; }
PK_ROWS_LDS=1 timeout -k 10 200 python -u tools/lin_bench.py > gpurun_out/$T/lin_bench_lds.txt 2>&1 || { cat gpurun_out/$T/lin_bench_lds.txt; exit 1; }
paste gpurun_out/$T/lin_bench.txt gpurun_out/$T/lin_bench_lds.txt
timeout -k 10 300 python -u bench.py --mode infer --no-cpu-baseline > gpurun_out/$T/infer.json 2> gpurun_out/$T/infer.err || exit $?
python3 -c "import json;d=json.loads(open('gpurun_out/$T/infer.json').read().strip().splitlines()[-1]);print('infer', d['value'], d['ms_per_step'], d['roofline'], {k: v['avg_ms'] for k, v in d['kernels'].items() if 'rigid' in k or 'ransac' in k})"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/prof_train -o run -- python3 bench.py --no-cpu-baseline --no-roofline-probe --train-only --steps 20 > gpurun_out/$T/prof_train.json 2> gpurun_out/$T/prof_train.err || exit $?
python3 tools/kstats.py gpurun_out/$T/prof_train/run_kernel_stats.csv 28 | head -45
