set -o pipefail
mkdir -p gpurun_out/r04c
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_configs_gpu.py -k "feat_dist or infer_step" -x -q --timeout 200 --timeout-method thread > gpurun_out/r04c/tests.log 2>&1 || { tail -30 gpurun_out/r04c/tests.log; exit 1; }
tail -3 gpurun_out/r04c/tests.log
timeout -k 10 200 python -u tools/fd_bench.py 20 "" fp32 > gpurun_out/r04c/fd_fused.txt 2>&1 || exit 1
PK_DEV=1 PK_FD_FUSED=0 timeout -k 10 200 python -u tools/fd_bench.py 20 "" fp32 > gpurun_out/r04c/fd_twopass.txt 2>&1 || exit 1
cat gpurun_out/r04c/fd_fused.txt gpurun_out/r04c/fd_twopass.txt
