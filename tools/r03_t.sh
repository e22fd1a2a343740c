export TMPDIR=/tmp
T=${TAG:-r03t}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u tools/glue_trace.py gpurun_out/$T/glue.txt > gpurun_out/$T/glue.log 2>&1 || { tail -30 gpurun_out/$T/glue.log; exit 1; }
cat gpurun_out/$T/glue.txt
