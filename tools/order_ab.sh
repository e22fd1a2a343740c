#!/bin/bash
# Overlapped training step: host enqueue order, queue priorities and the IR placement, alternating.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-orderab}
mkdir -p $O
i=0
for rep in 1 2; do
  for v in "" "--side-after" "--main-priority 1" "--main-priority -1" "--ir-main"; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 $v > $O/b_$i.log 2>&1 || { tail -20 $O/b_$i.log; exit 1; }
    grep "^{\"metric\"" $O/b_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$v] rep=$rep', d['value'], d['ms_per_step'])"
  done
done
