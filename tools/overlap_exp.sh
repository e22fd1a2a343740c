# Crop-formation overlap experiments: FPS variants (kbench fps), then the headline bench with the
# crop-formation stream on its own CUs (PK_SIDE_CUS) vs shared CUs, and the training stream alone.
export TMPDIR=/tmp
set -e
OUT=gpurun_out/ovl
mkdir -p $OUT
timeout -k 10 120 python tools/kbench.py fps > $OUT/kbench_fps.txt 2>&1
cat $OUT/kbench_fps.txt
for cus in 0 16 32; do
  PK_SIDE_CUS=$cus timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-probe --probe-steps 0 \
    > $OUT/bench_side$cus.json 2> $OUT/bench_side$cus.err
  python -c "import json;d=json.loads(open('$OUT/bench_side$cus.json').read().strip().splitlines()[-1]);print('side_cus=$cus', d['value'], d['ms_per_step'])"
done
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline-probe --probe-steps 0 --train-only \
  > $OUT/bench_trainonly.json 2> $OUT/bench_trainonly.err
python -c "import json;d=json.loads(open('$OUT/bench_trainonly.json').read().strip().splitlines()[-1]);print('train-only', d['value'], d['ms_per_step'])"
