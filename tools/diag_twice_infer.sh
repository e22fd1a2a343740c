# Marginal cost of crop-formation kernels beside the overlapped inference step (dev PK_DIAG_TWICE), alternating
export TMPDIR=/tmp
O=gpurun_out/${TAG:-diagtwinf}
mkdir -p $O
for rep in 1 2; do
  for v in none fps sorknn; do
    PK_DEV=1 PK_DIAG_TWICE=$v timeout -k 10 200 python bench.py --mode infer --steps 30 --warmup 5 --no-cpu-baseline --no-roofline-probe > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    grep "^{\"metric\"" $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('infer twice=$v rep=$rep', d['value'], d['ms_per_step'])"
  done
done
