# channels-first points-per-lane cap on the other lines (dev PK_CF_SUBMAX 4 = shipped, 1), alternating
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cfsub2}
mkdir -p $O
for rep in 1 2; do
  for args in "--mode infer" "--mode infer --points 2048" "--ragged --steps 10 --warmup 3"; do
    for v in 4 1; do
      PK_DEV=1 PK_CF_SUBMAX=$v timeout -k 10 300 python bench.py $args --no-cpu-baseline --no-roofline-probe > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
      grep "^{\"metric\"" $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('[$args] submax=$v rep=$rep', d['value'], d['ms_per_step'])"
    done
  done
done
