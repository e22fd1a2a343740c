#!/bin/bash
# round-4 batch 11: the weight-gradient pipeline kernel per shape group (kernel-trace durations).
export TMPDIR=/tmp
O=gpurun_out/r04b11
mkdir -p $O
for g in 0 1 2 3 4 5 6 7 8; do
  WG_ONLY=$g timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g$g -o run -- python3 -u tools/wg_bench.py 10 > $O/g$g.log 2>&1 || exit 1
  echo "$(grep -h '^group' $O/g$g.log) $(find $O/g$g -name '*kernel_stats.csv' | xargs grep -h wgrad_glds | cut -d, -f2-4)"
  find $O/g$g -type f ! -name "*stats.csv" -delete
done
