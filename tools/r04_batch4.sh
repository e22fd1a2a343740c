#!/bin/bash
# round-4 batch 4: feature-distance selection variants (AGPR accumulators, med3 forms) and PMC
# passes (MFMA busy / co-execution / VALU issue) for the FD kernel and the rigidity pair kernels.
export TMPDIR=/tmp
O=gpurun_out/r04b4
mkdir -p $O
VARS="0 1 5 7 8 9" TAG=r04b4/fd bash tools/fd_var.sh || exit 1
C1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for v in 0 1; do
  PK_DEV=1 PK_FD_VAR=$v timeout -s KILL 90 rocprofv3 --pmc $C1 --output-format csv -d $O/fdpmc$v -o run -- \
    python3 tools/fd_bench.py 5 32x1024 fp32 > $O/fdpmc$v.log 2>&1 || { tail -5 $O/fdpmc$v.log; exit 1; }
done
RIGID_ITERS=2 timeout -s KILL 120 rocprofv3 --pmc $C1 --output-format csv -d $O/rgpmc -o run -- \
  python3 tools/rigid_bench.py 2048 > $O/rgpmc.log 2>&1 || { tail -5 $O/rgpmc.log; exit 1; }
PK_DEV=1 PK_FD_VAR=0 timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES --output-format csv -d $O/fdco -o run -- \
  python3 tools/fd_bench.py 5 32x1024 fp32 > $O/fdco.log 2>&1 || { tail -5 $O/fdco.log; exit 1; }
echo done
