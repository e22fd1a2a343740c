"""Dev diagnostic: capture the training step (crop formation + forward_backward + clip +
RMSprop) into a HIP graph WITHOUT replaying it, dump the graph as DOT and list node
types, naming every memset / memcpy node and its neighbours (memset nodes were seen to
mis-order on replay on this stack, so the captured step must contain none).

  python tools/graph_dump.py [tag]
"""
import collections
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd.dataset.object import CropFormation  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402
from dpfm_amd.pipeline import TrainStep, make_frame_batch  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "gdump"
out = os.path.join(ROOT, "gpurun_out", tag)
os.makedirs(out, exist_ok=True)
dev = torch.device("cuda:0")
F_, N = 4, 512
fb, op = make_frame_batch(F_, N, N, seed=90, device=dev)
cf = CropFormation(n1=N, npoint=N, seed=1)
torch.manual_seed(0)
step = TrainStep(DPFMNet().to(dev), seed=5, capturable=True)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(2):
        step.forward_backward(op, cf(fb))
        step.apply()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
g.enable_debug_mode()
with torch.cuda.graph(g):
    step.forward_backward(op, cf(fb))
    step.apply(allreduce=False, reset=False)
path = os.path.join(out, "train_step_graph.dot")
try:
    g.debug_dump(path)
    txt = open(path).read()
except Exception as e:  # ROCm builds may not write the DOT file; use the API trace instead
    print("no DOT dump:", e)
    txt = ""
labels = re.findall(r'label="([^"]*)"', txt)
kinds = collections.Counter()
odd = []
for lab in labels:
    low = lab.lower()
    k = "kernel" if ("kernel" in low or "_z" in low) else ("memset" if "memset" in low else
                                                        ("memcpy" if "memcpy" in low else "other"))
    kinds[k] += 1
    if k in ("memset", "memcpy"):
        odd.append(lab[:300])
print("node kinds:", dict(kinds))
print("memset/memcpy nodes:", len(odd))
for o in odd[:40]:
    print("  ", o.replace("\\n", " | "))
