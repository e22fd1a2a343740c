#!/bin/bash
# Overlapped training step with crop formation on a reserved CU set (PipelinedTrainer side_cus):
# alternating runs of --side-cus values, 20 timed steps each.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cusab}
mkdir -p $O
for rep in 1 2; do
  for c in ${CUS:-0 32 48 64}; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 0 --side-cus $c ${EXTRA} > $O/b_${c}_$rep.log 2>&1 || { tail -20 $O/b_${c}_$rep.log; exit 1; }
    grep "^{\"metric\"" $O/b_${c}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('side_cus=$c rep=$rep', d['value'], d['ms_per_step'])"
  done
done
