# model / pipeline parity after the glue removal, then the glue trace and the step profile
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05glue}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_model_gpu.py tests/test_pipeline_gpu.py tests/test_ragged_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 tools/glue_trace.py $O/glue.txt > /dev/null 2>&1 || exit 1
cat $O/glue.txt
TAG=${TAG:-r05glue} bash tools/r05_prof.sh
