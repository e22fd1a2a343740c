#!/bin/bash
# Alternating runs of the overlapped step with the crop-formation kernels' wave priority 0..3.
O=gpurun_out/prio; mkdir -p $O
for r in 1 2; do for p in 0 1 2 3; do
  PK_SIDE_PRIO=$p timeout -k 10 200 python3 -u tools/prio_ab.py --steps 40 --no-cpu-baseline --no-roofline-probe > $O/p$p.r$r.json 2> $O/p$p.r$r.err || { tail -5 $O/p$p.r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/p$p.r$r.json').read().strip().splitlines()[-1]); print('prio $p run $r', d['value'], d['ms_per_step'])"
done; done
