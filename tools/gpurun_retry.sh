#!/bin/bash
# Re-submit a gpurun call only while the pool reports that nothing ran (exit 3, or a "transient"
# status: no box, busy slots, a box lost before the command started); any other outcome
# (including a failing command) is returned as is. When gpurun says it is backing off, wait the
# time it names before the next attempt.
# usage: tools/gpurun_retry.sh <timeout_s> '<command>'
T=$1; shift
log=$(mktemp)
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1 | tee "$log"
  rc=${PIPESTATUS[0]}
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$log"; then rm -f "$log"; exit $rc; fi
  wait_s=$(grep -o "retry in [0-9]*s" "$log" | grep -o "[0-9]*" | tail -1)
  wait_s=${wait_s:-60}
  echo "[retry] nothing ran (attempt $i); sleeping $((wait_s + 5)) s" >&2
  sleep $((wait_s + 5))
done
rm -f "$log"
exit 3
