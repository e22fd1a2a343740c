export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03d_model.log 2>&1; rc=$?
tail -5 gpurun_out/r03d_model.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python tools/lin_bench.py > gpurun_out/lin_bench_lds.txt 2>&1 || exit $?
PK_ROWS_ROUND2=1 timeout -k 10 200 python tools/lin_bench.py > gpurun_out/lin_bench_r2.txt 2>&1 || exit $?
paste gpurun_out/lin_bench_r2.txt gpurun_out/lin_bench_lds.txt | grep -v amdgpu
exit $rc
