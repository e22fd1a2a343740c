export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/pmc/avail.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p1 -o run -- python tools/fd_bench.py 5 32x1024 fp32 > gpurun_out/pmc/p1.log 2>&1
