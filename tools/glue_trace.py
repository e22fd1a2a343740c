"""Which torch ops (copies, adds, fills, cats) run outside libposekern in one eager training step,
and where they come from: a TorchDispatchMode logs each such aten op with its shapes / strides
and the innermost dpfm_amd Python frame (backward ops of built-in autograd nodes have none:
'engine'). python tools/glue_trace.py [out_file]"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

from dpfm_amd.dataset.object import CropFormation  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402
from dpfm_amd.pipeline import TrainStep, make_frame_batch  # noqa: E402

WATCH = ("copy_", "add", "add_", "cat", "fill_", "zero_", "zeros", "zeros_like", "new_zeros", "mean", "sum", "clone",
         "contiguous", "mul", "sub", "where", "any", "gt", "lt", "ne", "eq", "index", "stack", "neg", "div",
         "slice_backward", "select_backward", "threshold_backward", "split_backward", "_to_copy", "fill")
log = collections.Counter()


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in WATCH:
            t = [a for a in args if isinstance(a, torch.Tensor)]
            t += [x for a in args if isinstance(a, (list, tuple)) for x in a if isinstance(x, torch.Tensor)]
            if t and t[0].is_cuda:
                fr = [f for f in traceback.extract_stack() if "dpfm_amd" in f.filename]
                where = f"{os.path.basename(fr[-1].filename)}:{fr[-1].lineno} {fr[-1].name}" if fr else "engine"
                desc = " ".join(f"{tuple(x.shape)}/{tuple(x.stride())}" for x in t[:2])
                log[(name, desc, where)] += 1
        return func(*args, **(kwargs or {}))


dev = torch.device("cuda:0")
torch.manual_seed(1234)
model = DPFMNet().to(dev)
fb, op = make_frame_batch(32, 1024, 1024, seed=0, device=dev)
crops_of = CropFormation(n1=1024, npoint=1024, seed=0)
step = TrainStep(model, seed=0)
crops = crops_of(fb)
for _ in range(2):
    step(op, crops)
torch.cuda.synchronize()
with Mode():
    crops = crops_of(fb)  # crop formation (the timed step forms the next batch's crops beside it)
    step(op, crops)
torch.cuda.synchronize()
out = sys.argv[1] if len(sys.argv) > 1 else None
lines = [f"{n:3d}  {k[0]:10s} {k[2]:45s} {k[1]}" for k, n in sorted(log.items(), key=lambda kv: kv[0][2])]
txt = "\n".join(lines)
print(txt)
if out:
    open(out, "w").write(txt + "\n")
