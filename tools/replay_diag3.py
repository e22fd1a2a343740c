"""Dev diagnostic: crop formation captured in a HIP graph and replayed several times;
every intermediate of every stage compared with replay 0 (valid rows only), for the
ball-query mask kernel variants. Only libposekern + a few torch ops run (no model).

  python tools/replay_diag3.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

from dpfm_amd import _lib, ops  # noqa: E402
_lib.use_dev_lib()  # pkdev_* hooks: libposekern_dev.so (Makefile)
from dpfm_amd.pipeline import make_frame_batch  # noqa: E402

dev = torch.device("cuda:0")
F_, N = 4, 512
fb, op = make_frame_batch(F_, N, N, seed=90, device=dev)
L = _lib.lib()
L.pkdev_ball_query_mask_v1.argtypes = _lib.SIGNATURES["pk_ball_query_mask"]
_orig_call = _lib.call


def form(with_mask):
    bp = ops.backproject(fb.depth, fb.mask, fb.K, fb.cam_scale, cap=F_ * fb.max_pixels)
    so = ops.sor(bp["xyz"], bp["off"], fb.max_pixels, 20, 0.3, pix=bp["pix"], idxmap=bp["idxmap"], K=fb.K)
    pol = ops.fps_npoint(so["off"], fixed=N, limit=2000, seed=1)
    idx = ops.fps_packed(so["xyz32"], so["off"], fb.max_pixels, pol["start"], pol["npoint"], N)
    g = ops.gather_transform(so["xyz64"], so["off"], idx, pol["npoint"], N, pol["off"], fb.R, fb.t, F_ * N)
    bq = ops.ball_query(fb.cad64, fb.cad_off, g["align"], pol["off"], None, N, N, 64 * N, with_mask=with_mask,
                        thr2=fb.thr2)
    return dict(bp_count=bp["count"], bp_off=bp["off"], so_off=so["off"], so_avg=so["avg"], npoint=pol["npoint"],
                start=pol["start"], fps_idx=idx, align=g["align"], rowcount=bq["rowcount"], count=bq["count"],
                pairs=bq["pairs"], ov12=bq["overlap_12"], ov21=bq["overlap_21"],
                mask=bq["mask"] if with_mask else bq["rowcount"])


def run(label, with_mask, v1=False):
    if v1:
        def patched(name, *args, work=None):
            if name == "pk_ball_query_mask":
                st = L.pkdev_ball_query_mask_v1(*args)
                if st != 0:
                    raise RuntimeError(st)
                return
            return _orig_call(name, *args, work=work)
        ops.call = patched
    else:
        ops.call = _orig_call
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            form(with_mask)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    eager = {k: v.clone() for k, v in form(with_mask).items()}
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = form(with_mask)
    cap = out["pairs"].shape[1]
    for r in range(4):
        g.replay()
        torch.cuda.synchronize()
        cur = {k: v.clone() for k, v in out.items()}
        valid = torch.arange(cap, device=dev)[None] < torch.clamp(cur["count"], max=cap)[:, None]
        cur["pairs"] = cur["pairs"] * valid[..., None]
        ref = dict(eager)
        ref["pairs"] = ref["pairs"] * (torch.arange(cap, device=dev)[None] <
                                       torch.clamp(ref["count"], max=cap)[:, None])[..., None]
        bad = [k for k in ref if not torch.equal(ref[k], cur[k])]
        extra = ""
        if "ov21" in bad:
            d = (ref["ov21"] != cur["ov21"]).nonzero()
            extra = f" ov21 diffs {d.shape[0]} first {d[:4].tolist()} vals {cur['ov21'][d[:4, 0], d[:4, 1]].tolist()}"
        print(f"{label} replay {r}: {'OK' if not bad else 'DIFF ' + ','.join(bad)}{extra}", flush=True)


run("mask(stream)", True)
run("nomask(stream)", False)
run("mask(v1)", True, v1=True)
print("done")
