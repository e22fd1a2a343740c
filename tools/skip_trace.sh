# Step-window traces of the overlapped training step under diagnostic variants (head-of-replay
# timing): $1 = tag, then "ENV=VAL ..." variant strings, each traced once
export TMPDIR=/tmp
O=gpurun_out/$1; shift; mkdir -p $O
i=0
for v in "$@"; do
  i=$((i+1))
  ( export $v; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr$i -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline-probe --probe-steps 0 > $O/b$i.log 2>&1 ) || exit 1
  grep '^{"metric"' $O/b$i.log | tail -1 > $O/b$i.json
  python tools/step_window_summary.py $(find $O/tr$i -name "*kernel_trace.csv" | head -1) $O/b$i.json > $O/sws$i.txt 2>&1
  find $O/tr$i -type f -delete
  echo "== $v"; head -1 $O/sws$i.txt; sed -n '/^queue 1/,/^queue 4/p' $O/sws$i.txt | head -4; sed -n '/^queue 4/,$p' $O/sws$i.txt | head -26 | grep -v "^ *$"
done
