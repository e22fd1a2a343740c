set -u
mkdir -p gpurun_out/exp1
for cfg in "none 0" "aux 0" "side 0" "all 0" "none 1" "all 1"; do
  set -- $cfg
  PK_STEP_OVERLAP=$1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=$2 timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline-probe --probe-steps 1 > gpurun_out/exp1/b_$1_$2.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/exp1/b_$1_$2.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/exp1/b_$1_$2.log').read().strip().splitlines()[-1]);print('$cfg',d['value'],d['ms_per_step'])"
done
