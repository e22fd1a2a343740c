#!/bin/bash
# Re-submit a gpurun call only while the pool reports "no box / transient" (exit 3, nothing
# charged, nothing ran); any other outcome (including a failing command) is returned as is.
# usage: tools/gpurun_retry.sh <timeout_s> '<command>'
T=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] pool transient (exit 3), attempt $i; sleeping 60 s" >&2
  sleep 60
done
exit 3
