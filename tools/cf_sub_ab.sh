# channels-first layers: points per lane capped (dev PK_CF_SUBMAX: 4 = shipped choice, 1 = 16 points per wave), alternating
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cfsub}
mkdir -p $O
for rep in 1 2; do
  for v in 4 1; do
    PK_DEV=1 PK_CF_SUBMAX=$v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline-probe > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
    grep "^{\"metric\"" $O/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('submax=$v rep=$rep', d['value'], d['ms_per_step'])"
  done
done
for v in 4 1; do
  PK_DEV=1 PK_CF_SUBMAX=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k$v -o run -- python bench.py --train-only --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/k$v.log 2>&1 || exit 1
  f=$(find $O/k$v -name "*kernel_stats.csv" | head -1)
  echo "submax=$v cf kernels (train only):"; grep -E "linear_fwd_cf|linear_cf_pair" $f | python3 -c "
import sys,csv
t=0
for r in csv.reader(sys.stdin):
    t+=float(r[2]); print('  ', r[0][:60], r[1], round(float(r[3])/1e3,2))
print('  total ms', round(t/1e6,3))"
  find $O/k$v -type f ! -name "*kernel_stats.csv" -delete
done
