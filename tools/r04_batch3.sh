#!/bin/bash
# round-4 batch 3: weight-gradient pipeline (cost-balanced slices, adaptive ring) tests + census,
# rigidity (scalar FMA pair term) tests + A/B, feature-distance limiter variants, and the
# inference bench at 2048 points with a kernel trace (per-round rigidity times).
export TMPDIR=/tmp
O=gpurun_out/r04b3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_configs_gpu.py -x -q \
  --timeout 200 --timeout-method thread -k "wgrad or graphed or pipelined or train_and_infer or rigid or chain" > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/lin_census.py > $O/census.txt 2>&1 || { tail $O/census.txt; exit 1; }
grep -A12 "pk_linear_wgrad_grouped" $O/census.txt
timeout -k 10 200 python3 -u tools/rigid_bench.py 1024 2048 > $O/rigid.txt 2>&1 || { tail $O/rigid.txt; exit 1; }
cat $O/rigid.txt
TAG=r04b3/fd bash tools/fd_var.sh || exit 1
timeout -k 10 300 python3 -u bench.py --mode infer --points 2048 --no-cpu-baseline > $O/infer2048.json 2> $O/infer2048.err || { tail $O/infer2048.err; exit 1; }
cat $O/infer2048.json | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ikt -o run -- python3 -u bench.py --mode infer --points 2048 --no-cpu-baseline --steps 3 --warmup 1 --no-roofline-probe > $O/ikt.log 2>&1 || exit 1
