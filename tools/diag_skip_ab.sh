#!/bin/bash
# How much each crop-formation kernel's occupancy costs the overlapped training step: the dev
# library's PK_DIAG_SKIP leaves the named launches out (timing diagnostic only; the crops are
# then garbage), alternating runs.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-diagskip}
mkdir -p $O
i=0
for rep in 1 2; do
  for v in none fps sorknn fps,sorknn; do
    i=$((i+1))
    PK_DEV=1 PK_DIAG_SKIP=$v timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/b_$i.log 2>&1 || { tail -20 $O/b_$i.log; exit 1; }
    grep "^{\"metric\"" $O/b_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('skip=$v rep=$rep', d['value'], d['ms_per_step'])"
  done
done
