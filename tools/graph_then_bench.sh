#!/bin/bash
# Validate HIP-graph capture piece by piece (tools/graph_diag.py) before anything runs a
# captured step; only on a clean pass go on to the tests and benches. A diagnostic
# mismatch (exit 1, no fault) retries the diagnostic with rocBLAS as the BLAS backend.
tag=$1
tools/gpu_run.sh "$tag" gdiag
rc=$?
if [ $rc -eq 0 ]; then
  tools/gpu_run.sh "$tag" tests benchq benche prof pmc
  exit $?
elif [ $rc -eq 1 ]; then
  tools/gpu_run.sh "${tag}b" gdiag_rocblas
  exit $?
fi
exit $rc
