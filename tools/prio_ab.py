"""A/B of the crop-formation kernels' wave priority (PK_SIDE_PRIO, common.hpp side_prio): runs
bench.py's overlapped training step through libposekern_dev.so, which reads the variable.

  PK_SIDE_PRIO=2 python3 tools/prio_ab.py --steps 40 --no-cpu-baseline --no-roofline-probe
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from dpfm_amd import _lib  # noqa: E402

_lib.use_dev_lib()
sys.argv = [sys.argv[0]] + sys.argv[1:]
bench.main()
