#!/bin/bash
# Counter record of the shipped feature-distance kernels (profiles/r06_fd_pmc.txt): one rocprofv3
# pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, SQ_INSTS_VALU, SQ_INSTS_MFMA,
# GRBM_GUI_ACTIVE) over tools/fd_bench.py at configs[1] (32 x 1024 x 1024, fp32, top-1 and top-5),
# then the same calls timed without counters, and the inference bench line.
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06fdpmc}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o run -- python tools/fd_bench.py 5 32x1024 fp32 1,5 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python tools/mfma_util.py $O/pmc fd_top1_kernel fd_top1_prep_kernel fd_top5_kernel fd_merge_kernel > $O/mfma_util.json 2>&1
find $O/pmc -type f -name "*.csv" ! -name "*counter_collection.csv" -delete
timeout -k 10 200 python tools/fd_bench.py 20 32x1024 fp32 1,5 > $O/fdb.log 2>&1 && grep -v amdgpu $O/fdb.log
timeout -k 10 300 python bench.py --mode infer > $O/infer.log 2>&1 && grep "^{\"metric\"" $O/infer.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('infer', d['value'], d['ms_per_step']); print(d['roofline_mfma_kernels']); print({k: v for k, v in d['kernels'].items() if 'feat' in k})"
cat $O/mfma_util.json | head -60
