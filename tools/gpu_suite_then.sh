# Full -m gpu suite, then an optional follow-up script, stopping on a GPU fault / abort /
# segfault / time limit of the suite (exit 124, 134, 137, 139) and running the follow-up only
# after a clean or ordinarily failing (assertion) suite run.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --durations=15 --timeout 600 --timeout-method thread \
  > gpurun_out/${TAG:-r03}_gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/${TAG:-r03}_gpu_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
if [ -n "$1" ]; then bash "$@" || exit $?; fi
exit $rc
