#!/bin/bash
# Alternating runs of the overlapped step with C_gt and / or the IR moved from the crop-formation
# stream into the training graph (bench.py --cgt-main / --ir-main).
O=gpurun_out/side_ab; mkdir -p $O
for r in 1 2; do for v in "" "--cgt-main" "--ir-main" "--cgt-main --ir-main"; do
  n=$(echo "x$v" | tr -d ' -'); 
  timeout -k 10 200 python3 -u bench.py --steps 40 --no-cpu-baseline --no-roofline-probe $v > $O/$n.r$r.json 2> $O/$n.r$r.err || { tail -5 $O/$n.r$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.r$r.json').read().strip().splitlines()[-1]); print('[$v] run $r', d['value'], d['ms_per_step'])"
done; done
