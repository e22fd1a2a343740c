# round-5 FD iteration: bench (prep + main, and the dev one-launch form), stamps, FD tests
mkdir -p gpurun_out/r05
for sh in 32x1024 8x2048 1x4096; do timeout -k 10 120 python3 -u tools/fd_bench.py 20 $sh fp32 2>&1 | grep feat_dist || exit 1; done
PK_DEV=1 PK_FD_VAR=20 timeout -k 10 120 python3 -u tools/fd_bench.py 20 32x1024 fp32 2>&1 | grep feat_dist | sed 's/^/[one-launch dev] /' || exit 1
PK_DEV=1 PK_FD_VAR=13 timeout -k 10 120 python3 -u tools/fd_stamps.py 32x1024 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python3 -u -m pytest tests/test_configs_gpu.py tests/test_corr_pose_gpu.py -k "feat_dist or naive" -x -q --timeout 120 --timeout-method thread -m gpu 2>&1 | tail -2
