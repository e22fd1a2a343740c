# ball-query mask probe, per-block fractions in time order (PK_BQ_VAR: 0 nt stores, 1 plain)
mkdir -p gpurun_out/r06bqab
for v in ${VARS:-0}; do PK_DEV=1 PK_BQ_VAR=$v timeout -k 10 120 python tools/bq_bench.py ${BLOCKS:-20} ${REPS:-2} > gpurun_out/r06bqab/v$v.log 2>&1 || exit 1; echo "var $v"; grep kernel gpurun_out/r06bqab/v$v.log | python3 -c "import sys,json; [print(json.loads(l)['frac'], json.loads(l)['frac_min'], json.loads(l)['frac_max'], json.loads(l)['frac_blocks']) for l in sys.stdin]"; done
