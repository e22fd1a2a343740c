# feature-distance parity subset, then top-1 / top-5 timings (graph, warmed) and top-5 phase stamps
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -k "feat_dist or top5 or infer_step" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/fd_bench.py 20 32x1024 fp32 1,5 > $O/fdb.log 2>&1 && grep -v amdgpu $O/fdb.log || exit 1
timeout -k 10 200 python tools/fd_bench.py 20 1x4096 fp32 1,5 > $O/fdb4096.log 2>&1 && grep -v amdgpu $O/fdb4096.log || exit 1
PK_DEV=1 PK_FD_VAR=13 timeout -k 10 120 python tools/fd_stamps.py 32x1024 5 > $O/t5.log 2>&1 && grep -v amdgpu $O/t5.log
PK_DEV=1 PK_FD_VAR=13 timeout -k 10 120 python tools/fd_stamps.py 32x1024 1 > $O/t1.log 2>&1 && grep -v amdgpu $O/t1.log
