#!/bin/bash
# A/B of CLR graph packet capture (DEBUG_CLR_GRAPH_PACKET_CAPTURE 0 = off, the default set by
# dpfm_amd; 1 = CLR's own default): host enqueue cost per training step, the bench step, and the
# graph-vs-eager bit-equality tests with capture on (a skipped memset node would break them).
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pcab}
mkdir -p $O
for pc in 0 1; do
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 300 python tools/host_launch.py > $O/host_$pc.log 2>&1 || { tail -20 $O/host_$pc.log; exit 1; }
  DEBUG_CLR_GRAPH_PACKET_CAPTURE=$pc timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline-probe > $O/bench_$pc.log 2>&1 || { tail -20 $O/bench_$pc.log; exit 1; }
  grep "^{\"metric\"" $O/bench_$pc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pc=$pc', d['value'], d['ms_per_step'])"
  grep "host enqueue" $O/host_$pc.log
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pipe_pc1.log 2>&1; echo "pipeline tests pc=1 rc=$?"; tail -3 $O/pipe_pc1.log
