#!/bin/bash
# The round-6 FPS chain trims (production) against the round-5 chain (dev PK_FPS_TRIM=0) in the
# overlapped training and inference steps, alternating runs on one box, unprofiled.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fpstrim}
mkdir -p $O
PK_FPS_TRIM=0 KB_FAST=1 timeout -k 10 200 python -u tools/kbench.py fps > $O/kbench_untrimmed.txt 2>&1 || exit 1
tail -3 $O/kbench_untrimmed.txt
i=0
for rep in 1 2 3; do
  for mode in train infer; do
    for v in 0 1; do
      i=$((i+1))
      PK_DEV=1 PK_FPS_TRIM=$v timeout -k 10 200 python bench.py --mode $mode --steps 30 --warmup 5 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/b_$i.log 2>&1 || { tail -20 $O/b_$i.log; exit 1; }
      grep "^{\"metric\"" $O/b_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode trim=$v rep=$rep', d['value'], d['ms_per_step'])"
    done
  done
done
