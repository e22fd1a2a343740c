"""CPU oracle for the RGB-D pose hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package, and only as the checker / CPU baseline. The product path
(6d-pose-estimation-for-unseen-categories_amd/dpfm_amd) never imports it and fails
loudly when its HIP library is missing.

Contents
  dpfm_oracle.py  literal numpy / torch-CPU restatements of the reference lines
                  (each function cites the /root/reference file:line it follows)
  c/oracle.c      plain-C restatements of the sequential / O(n^2) kernels (FPS,
                  ball query, Umeyama + RANSAC) used for big-size parity and as the
                  timed CPU baseline (kind "port")

Pinning status: the reference cannot be imported here
(environment denial recorded in SURVEY.md §8(c)) and has no tests. Pose metrics
(H14) are pinned against the reference's own published per-crop outputs
(results_on_*/…/results/*.txt + ply) by tests/golden/make_golden.py; every other
row is a literal restatement whose parity is unpinned against the reference
itself (third-party code — DPFM submodule, Open3D, OpenCV — is absent).
"""
