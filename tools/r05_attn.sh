# attention backward (one-pass) parity + the model / pipeline tests that run through it, then the step profile
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05attn}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_ragged_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r05attn} bash tools/r05_prof.sh
