export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ncep/$1 -o run -- python tools/nce_bench.py > /dev/null 2>&1
find gpurun_out/ncep/$1 -type f ! -name "*kernel_stats.csv" -delete
cut -d, -f1-4 gpurun_out/ncep/$1/run_kernel_stats.csv | grep -i "nce\|zero" | cut -c1-60,150-260
