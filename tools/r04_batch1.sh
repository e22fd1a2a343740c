#!/bin/bash
# round-4 batch: layer + feature-distance + rigidity tests, then the layer A/B, the
# feature-distance variants and the rigidity A/B with a kernel trace.
export TMPDIR=/tmp
O=gpurun_out/r04b1
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_configs_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "linear or encoder or dpfmnet or relu or block or overlap or attn_prop or feat_dist or rigid or chain" \
  > $O/tests.txt 2>&1
rc=$?; tail -5 $O/tests.txt; [ $rc -eq 0 ] || exit $rc
TAG=r04b1/lin bash tools/lin_ab.sh || exit 1
TAG=r04b1/fd bash tools/fd_var.sh || exit 1
timeout -k 10 200 python3 -u tools/rigid_bench.py 1024 2048 > $O/rigid.txt 2>&1 || { tail $O/rigid.txt; exit 1; }
cat $O/rigid.txt
RIGID_ITERS=5 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/rprof -o rp -- python3 -u tools/rigid_bench.py 2048 > $O/rigid_prof.txt 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/lin_census.py > $O/census.txt 2>&1 || { tail $O/census.txt; exit 1; }
tail -30 $O/census.txt
