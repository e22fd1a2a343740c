# round-5: FD bench + stamps, then the index-guard, feature-distance, pipeline and correspondence tests
mkdir -p gpurun_out/r05
rm -f gpurun_out/r05/fdbench.txt
for sh in 32x1024 8x2048 1x4096; do
  timeout -k 10 120 python3 -u tools/fd_bench.py 20 $sh fp32 2>&1 | grep feat_dist >> gpurun_out/r05/fdbench.txt || exit 1
done
cat gpurun_out/r05/fdbench.txt
PK_DEV=1 PK_FD_VAR=13 timeout -k 10 120 python3 -u tools/fd_stamps.py 32x1024 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python3 -u -m pytest tests/test_index_guard_gpu.py tests/test_configs_gpu.py tests/test_corr_pose_gpu.py tests/test_pipeline_gpu.py tests/test_crops_gpu.py tests/test_fps_ballquery_gpu.py tests/test_ragged_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r05/tests2.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05/tests2.log | tail -80
exit $rc
