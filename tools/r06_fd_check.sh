export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/fd_bench.py 20 32x1024 fp32 1,5 > $O/fdb.log 2>&1 && grep -v amdgpu $O/fdb.log
PK_FD_TOP5_OLD=1 PK_DEV=1 timeout -k 10 200 python tools/fd_bench.py 20 32x1024 fp32 5 > $O/fdb_old.log 2>&1 && grep -v amdgpu $O/fdb_old.log
bash tools/rt_trace.sh r06j/rt > /dev/null 2>&1; head -60 gpurun_out/r06j/rt/summary.txt
