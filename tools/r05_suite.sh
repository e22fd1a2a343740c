# full GPU suite, then the headline bench (train) and inference bench lines
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05suite}
mkdir -p $O
timeout -k 10 1500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $O/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u bench.py > $O/train.out 2> $O/train.err || { tail -20 $O/train.err; exit 1; }
tail -c 3000 $O/train.out
