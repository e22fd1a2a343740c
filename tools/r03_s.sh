export TMPDIR=/tmp
T=${TAG:-r03s}
mkdir -p gpurun_out/$T
for tk in 64 128; do
  PK_ATTN_FWD_TK=$tk timeout -k 10 120 python -u tools/attn_pmc.py 30 > gpurun_out/$T/attn$tk.txt 2>&1 || { cat gpurun_out/$T/attn$tk.txt; exit 1; }
  echo "tk=$tk $(tail -1 gpurun_out/$T/attn$tk.txt)"
  PK_ATTN_FWD_TK=$tk timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/tr$tk -o run -- python3 tools/attn_pmc.py 10 > gpurun_out/$T/tr$tk.log 2>&1 || exit 1
  python3 tools/kstats.py gpurun_out/$T/tr$tk/run_kernel_stats.csv | head -5
done
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q -k "attention or dpfm or fused" --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
