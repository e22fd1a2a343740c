#!/bin/bash
# round-4 batch 10: weight-gradient pipeline kernel time vs the block budget (dev PK_WG_BUDGET).
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04b10}
mkdir -p $O
for b in ${BUDGETS:-256 512 1024 128}; do
  PK_DEV=1 PK_WG_BUDGET=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/b$b -o run -- python3 -u tools/wg_bench.py 5 > $O/b$b.log 2>&1 || exit 1
  grep -h "device\|wgrad grouped" $O/b$b.log
  find $O/b$b -name "*kernel_stats.csv" | xargs cat | cut -d, -f1-4 | grep -i "wgrad"
  find $O/b$b -type f ! -name "*stats.csv" -delete
done
