"""Ball-query mask roofline probe alone (bench.ball_query_roofline at configs[3] size):
python tools/bq_bench.py [blocks] [repeats]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

blocks = int(sys.argv[1]) if len(sys.argv) > 1 else 7
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
if os.environ.get("PK_DEV") == "1":  # PK_BQ_VAR store-flavour A/B (tools/bq_ab.sh)
    from dpfm_amd import _lib
    _lib.use_dev_lib()
dev = torch.device("cuda:0")
for _ in range(reps):
    r = bench.ball_query_roofline(dev, blocks=blocks)
    r.pop("traffic", None)
    print(json.dumps(r), flush=True)
