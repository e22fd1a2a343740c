#!/bin/bash
# Weight-gradient pipeline limiter study (dev PK_WG_VAR): 0 production, 1 no MFMAs, 2 the glds stream alone;
# kernel time of wgrad_glds_grouped_kernel on the training step's call list (tools/wg_bench.py) under rocprofv3.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-wgvar}
mkdir -p $O
for v in 0 1 2; do
  PK_DEV=1 PK_WG_VAR=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$v -o run -- python3 -u tools/wg_bench.py 5 > $O/v$v.log 2>&1 || exit 1
  echo "var $v: $(find $O/v$v -name '*kernel_stats.csv' | xargs grep -h wgrad_glds | cut -d, -f2-4)"
  find $O/v$v -type f ! -name "*stats.csv" -delete
done
