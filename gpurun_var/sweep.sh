# swap each variant library in, time SOR standalone and the overlapped training step
L=6d-pose-estimation-for-unseen-categories_amd/dpfm_amd/lib/libposekern.so
cp $L gpurun_out/lib_orig.so
for v in gpurun_var/libposekern_*.so; do
  cp $v $L
  s=$(timeout -k 10 100 python tools/kbench.py fps 2>&1 | grep "^sor" | sed 's/.*: //')
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-roofline-probe --probe-steps 0 $1 > gpurun_out/bv.json 2>gpurun_out/bv.err || { cp gpurun_out/lib_orig.so $L; exit 1; }
  echo "$(basename $v) sor: $s | step $(tail -1 gpurun_out/bv.json | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d[\"ms_per_step\"])")"
done
cp gpurun_out/lib_orig.so $L
rm gpurun_out/lib_orig.so
