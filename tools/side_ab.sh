#!/bin/bash
# Alternating runs of the overlapped step with C_gt on the crop-formation stream (--cgt-side;
# default: in the training graph) and / or the IR in the training graph (--ir-main).
O=gpurun_out/side_ab; mkdir -p $O
for r in 1 2; do for v in "" "--cgt-side 1" "--ir-main" "--cgt-side 1 --ir-main"; do
  n=$(echo "x$v" | tr -d ' -'); 
  timeout -k 10 200 python3 -u bench.py --steps 40 --no-cpu-baseline --no-roofline-probe $v > $O/$n.r$r.json 2> $O/$n.r$r.err || { tail -5 $O/$n.r$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.r$r.json').read().strip().splitlines()[-1]); print('[$v] run $r', d['value'], d['ms_per_step'])"
done; done
