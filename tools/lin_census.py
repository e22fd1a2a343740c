"""Census of the training step's per-point layer launches (pk_linear_ex): every call of one
eager probe step at configs[1] (bench.py's train build), grouped by shape and epilogue, with
HIP-event time per call and the algorithmic bytes (ops.linear_ex's `work`)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from dpfm_amd import _lib, ops  # noqa: E402

if os.environ.get("PK_DEV") == "1":  # libposekern_dev.so (its PK_* switches, e.g. PK_WG_GLDS=0)
    _lib.use_dev_lib()

sys.argv = ["bench.py"]
args = bench.parse()
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
one_step, probe_step, *_ = bench.build_train(args, dev, 0, 1)
for _ in range(3):
    one_step()
torch.cuda.synchronize()

calls = []
orig = ops.linear_ex


def rec(x, w, bias, layout, R, N, Cin, Cout, y, **kw):
    flags = [k for k in ("mask", "y2", "add", "pre", "w2", "add2") if kw.get(k) is not None]
    if kw.get("store_cf"):
        flags.append("store_cf")
    if kw.get("transw"):
        flags.append("T")
    if kw.get("relu") or kw.get("act"):
        flags.append(f"act{kw.get('act') if kw.get('act') is not None else 1}")
    calls.append(["cf" if layout else "cl", R, Cin, Cout, "+".join(flags)])
    return orig(x, w, bias, layout, R, N, Cin, Cout, y, **kw)


ops.linear_ex = rec
times = []
wcalls = []
orig_w = ops.linear_wgrad_grouped


def rec_w(cl):
    wcalls.append([("cf", tuple(x.shape), dy.shape[1]) if cf else ("cl", x.numel() // x.shape[-1], x.shape[-1],
                   dy.shape[-1]) for (x, dy, cf, dw, db, acc) in cl])
    return orig_w(cl)


ops.linear_wgrad_grouped = rec_w


def hook(name, fn, work=None):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    r = fn()
    e.record()
    if name == "pk_linear_ex":
        times.append((s, e, work))
    if name == "pk_linear_wgrad_grouped":
        wtimes.append((s, e, work))
    return r


wtimes = []
for rep in range(2):
    calls.clear()
    times.clear()
    wcalls.clear()
    wtimes.clear()
    _lib.set_probe(hook)
    torch.cuda.synchronize()
    torch.cuda._sleep(int(2.5e8))
    probe_step()
    torch.cuda.synchronize()
    _lib.set_probe(None)
assert len(calls) == len(times), (len(calls), len(times))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
for c, (s, e, w) in zip(calls, times):
    k = tuple(c)
    agg[k][0] += 1
    agg[k][1] += s.elapsed_time(e) * 1e3
    agg[k][2] += w[1]
tot = sum(v[1] for v in agg.values())
print(f"{len(calls)} pk_linear_ex calls, {tot:.1f} us per step")
for k, (n, us, byts) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{str(k):60s} n={n:2d} {us / n:6.1f} us/call {us:7.1f} us total  {byts / n / 1e6:6.2f} MB/call "
          f"{byts / (us * 1e-6) / 1e9:6.0f} GB/s")

for cl, (s, e, w) in zip(wcalls, wtimes):
    rows = collections.Counter(map(tuple, cl))
    print(f"pk_linear_wgrad_grouped: {len(cl)} calls, {s.elapsed_time(e) * 1e3:.1f} us, {w[1] / 1e9:.2f} GFLOP")
    for k, n in sorted(rows.items(), key=lambda kv: str(kv[0])):
        print(f"   {str(k):50s} x{n}")
