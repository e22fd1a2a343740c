# Operators (tufted Laplacian, new-crop chain) on the GPU, attention variants, torch glue profile.
export TMPDIR=/tmp
T=${TAG:-r03h}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_operators_gpu.py > gpurun_out/$T/tests.log 2>&1 || { tail -40 gpurun_out/$T/tests.log; exit 1; }
tail -2 gpurun_out/$T/tests.log
bash tools/attn_var.sh 2>&1 | tee gpurun_out/$T/attn_var.txt || exit 1
timeout -k 10 300 python -u tools/torch_prof.py $T > gpurun_out/$T/tprof.log 2>&1 || { tail -20 gpurun_out/$T/tprof.log; exit 1; }
head -40 gpurun_out/$T/torch_prof_glue.txt
