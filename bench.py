"""Headline benchmark: RGB-D crops/sec (fwd+bwd), 1024-point crops, per BASELINE.json.

One step = one training iteration of the reference (scripts/train.py:88-124) for a batch
of B synthetic 640x480 RGB-D frames, with the dataset's crop formation on the device:
  back-projection + erosion -> SOR kNN-20 -> FPS to 1024 -> align transform -> ball
  query (P, overlaps) -> DPFMNet fwd -> C_gt + DPFMLoss ->
  naive point map + inlier ratio -> backward -> grad all-reduce (N > 1) -> clip -> RMSprop.
Inputs (frames, CAD models, cached spectral operators) are resident in HBM before timing.

  python bench.py [--gpus N --steps K --warmup W --batch B]   (N > 1: spawns N ranks itself)
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
Rank 0 prints one JSON line (contract in the task statement / DESIGN.md §Measurement).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")  # see dpfm_amd/__init__.py (HIP-graph memset replays)

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
F32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 matrix (= vector) peak
F32_VALU_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector peak
F64_VALU_TFLOPS = 78.6    # AMD MI355X datasheet FP64 vector (not in the guide; half the FP32 vector rate)
BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense BF16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="crops per GPU (configs[1]: 32)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="crops over all ranks (per rank = global / N; configs[2]: --gpus 2 --global-batch 32); "
                         "default: --batch per GPU (weak scaling)")
    ap.add_argument("--points", type=int, default=1024)
    ap.add_argument("--ragged", action="store_true",
                    help="train / infer at the reference's real sizes: ragged crops of ~200-2000 points (the "
                         "object.py:145-148 sample policy), ~5000-vertex CADs, collate padding to 2000")
    ap.add_argument("--cad-points", type=int, default=5000, help="--ragged: CAD vertices")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-crops", type=int, default=30, help="bounded CPU-baseline sample (crops)")
    ap.add_argument("--pose-crops", type=int, default=8,
                    help="train: crops of the post-timing pose-vs-reference check (0: skip)")
    ap.add_argument("--no-roofline-probe", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP graph: launch every kernel from Python")
    ap.add_argument("--side-after", action="store_true",
                    help="train overlapped: enqueue each training replay before the next crop formation")
    ap.add_argument("--side-cus", type=int, default=0,
                    help="train/infer overlapped: crop formation on this many CUs, the step on the rest (0: shared)")
    ap.add_argument("--main-priority", type=int, default=0,
                    help="1: the training stream at the highest HIP queue priority (crop formation below)")
    ap.add_argument("--cgt-side", type=int, choices=(0, 1), default=None,
                    help="1: solve C_gt with the crops on the crop-formation stream, 0: in the training graph "
                         "(default: 0 for the configs[1] shape, 1 for --ragged: measured faster for each, DESIGN 5b)")
    ap.add_argument("--ir-main", action="store_true",
                    help="keep the naive point map + IR in the training graph (no deferred I_k graph)")
    ap.add_argument("--train-only", action="store_true",
                    help="diagnostic: crops formed once, outside the timed graph (not a headline number)")
    ap.add_argument("--infer-stages", type=int, choices=(2, 3), default=2,
                    help="infer: 3 = also overlap the pose stage of batch i-1 with the model of batch i")
    ap.add_argument("--no-overlap", action="store_true",
                    help="graph mode without overlapping crop formation of the next batch")
    ap.add_argument("--probe-steps", type=int, default=2, help="eager steps after timing for the kernel breakdown")
    ap.add_argument("--mode", choices=("train", "infer", "corr4096", "icp", "teaser", "operators", "ransac_ref"),
                    default="train",
                    help="train: the headline fwd+bwd step (default); infer: configs[1]/[3] inference; "
                         "corr4096: configs[4] feature distance + RANSAC; icp: the (f4) ICP refinement; "
                         "teaser: the (f2) TEASER++ solver; operators: the (f1) spectral operators")
    ap.add_argument("--op-points", type=int, default=2000, help="operators: points per crop")
    ap.add_argument("--icp-evals", type=int, default=0,
                    help="infer: refine every RANSAC pose by ICP against the crop (evaluations enqueued)")
    ap.add_argument("--teaser-n", type=int, default=2000, help="teaser: correspondences per crop")
    ap.add_argument("--icp-target", choices=("gt_cad", "crop"), default="gt_cad",
                    help="icp: the reference's target (CAD under T_gt) or the observed crop")
    ap.add_argument("--hypotheses", type=int, default=1024, help="RANSAC hypotheses per crop (infer/corr4096)")
    ap.add_argument("--ransac-crops", type=int, default=1, help="ransac_ref: crops per step")
    ap.add_argument("--fd-precision", choices=("fp32", "bf16", "bf16x3"), default="fp32",
                    help="corr4096: feature-distance contraction precision (fp32 = the parity path)")
    return ap.parse_args()


class KernelProbe:
    """HIP events around every libposekern call (same stream as the kernels: torch's
    current stream), with the algorithmic work each launch declares (ops.py `work=`)."""

    def __init__(self):
        self.ev = {}

    # entry points reported as one family: a pk_linear_ex2 call is two per-point layers in one
    # launch (one family launch, both layers' bytes)
    FAMILY = {"pk_linear_ex2": "pk_linear_ex"}

    def hook(self, name, fn, work=None):
        name = self.FAMILY.get(name, name)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = fn()
        e.record()
        self.ev.setdefault(name, []).append((s, e, work))
        return r

    def summary(self):
        """name -> dict(avg_ms, launches, total_ms, bound, work) (work summed, or None)."""
        out = {}
        for k, lst in self.ev.items():
            ms = [s.elapsed_time(e) for s, e, _ in lst]
            works = [w() if callable(w) else w for _, _, w in lst]  # deferred: read after the timed region
            known = all(w is not None for w in works)
            out[k] = dict(avg_ms=float(np.mean(ms)), launches=len(ms), total_ms=float(np.sum(ms)),
                          bound=works[0][0] if known else None,
                          work=float(sum(w[1] for w in works)) if known else None,
                          flops=float(sum(w[2] for w in works)) if known and all(len(w) > 2 for w in works) else None)
        return out


def ball_query_roofline(dev, probe_launches: int = 10, blocks: int = 7) -> dict:
    """pk_ball_query_mask at configs[3] size (B=256 crops, 2048 x 2048): >= 1 GB per launch.
    `blocks` timed blocks of `probe_launches` back-to-back launches each: the line reports the
    median block (achieved / frac) and the min / max over blocks (run-to-run spread)."""
    from dpfm_amd import ops
    from dpfm_amd._lib import call, ptr, stream
    B, N = 256, 2048
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    cad = torch.randn((B * N, 3), dtype=torch.float64, device=dev, generator=g) * 5
    pc = torch.randn((B * N, 3), dtype=torch.float64, device=dev, generator=g) * 5
    off = ops.packed_offsets([N] * B, dev)
    thr = torch.full((B,), ops.ball_threshold(0.6), dtype=torch.float64, device=dev)
    mask = torch.empty((B, N, N), dtype=torch.uint8, device=dev)
    rc = torch.empty((B, N), dtype=torch.int32, device=dev)
    f = lambda: call("pk_ball_query_mask", ptr(cad), ptr(off), ptr(pc), ptr(off), ptr(thr), B, N, N, ptr(mask), N,  # noqa
                     ptr(rc), stream(dev))
    # untimed warm-up, ~60 ms of launches: under this write load the clocks ramp for ~25 ms (the
    # per-block fractions climb 0.48 -> 0.62 over the first 10 blocks, profiles/r06_bq_ramp.txt)
    for _ in range(25 * probe_launches):
        f()
    torch.cuda.synchronize()
    byts = B * (24 * N + 24 * N + N * N) + B * N * 4  # coords in + mask + row counts
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(blocks)]
    for s, e in ev:
        s.record()
        for _ in range(probe_launches):
            f()
        e.record()
    torch.cuda.synchronize()
    seq = [s.elapsed_time(e) / probe_launches for s, e in ev]  # time order
    mss = sorted(seq)
    ms = float(np.median(mss))
    fr = lambda m: round(byts / (m * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)  # noqa: E731
    ach = byts / (ms * 1e-3) / 1e9
    return {"kernel": "pk_ball_query_mask (configs[3]: 256 x 2048 x 2048)", "bound": "hbm", "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "frac_min": fr(mss[-1]), "frac_max": fr(mss[0]), "frac_blocks": [fr(m) for m in seq],
            "blocks": blocks, "launches_per_block": probe_launches,
            "traffic": pmc_traffic("pk_ball_query_mask@configs3_probe"),
            "ms_per_launch": round(ms, 4), "bytes_per_launch": byts}


def feat_dist_roofline(dev, launches: int = 20, topk: int = 1) -> dict:
    """The north-star MFMA gate kernel: pk_feat_dist_topk (fp32 argmin, the naive solver's and the
    IR's feature distance, fmap2pointmap_solvers/naive.py:20,33) at configs[1] (32 crops of
    1024 x 1024, K = 32: 2.147 GFLOP per call), `launches` back-to-back calls in one HIP graph
    between two HIP events on the launch stream (its prep + main passes included), spectral-basis
    operands. topk=5: the configured solver's top-5 (spacial_filtering.py:19,32-38; the same
    contraction, its epilogue and near-tie recompute included in the time)."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import lbo_operators
    B, V = 32, 1024
    ex = torch.stack([torch.from_numpy(lbo_operators(V, 64, 10 + b)[2]) for b in range(B)]).to(dev)
    ey = torch.stack([torch.from_numpy(lbo_operators(V, 64, 50 + b)[2]) for b in range(B)]).to(dev)
    C = (torch.eye(30)[None] + 0.3 * torch.randn(B, 30, 30, generator=torch.Generator().manual_seed(B))).to(dev)
    n = torch.full((B,), V, dtype=torch.int32, device=dev)
    wk = torch.empty(1 << 24, dtype=torch.uint8, device=dev)
    f = lambda: ops.feat_dist_topk(ex, C, ey, n, n, topk, work=wk)  # noqa: E731
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    # the calls as the pipeline issues them (HIP graph: no host gaps), timed after ~60 ms of
    # replays (clock ramp, profiles/r06_bq_ramp.txt); median of 5 timed replays
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(launches):
            f()
    for _ in range(100):
        gr.replay()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for s, e in evs:
        s.record()
        gr.replay()
        e.record()
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in evs)[2] / launches
    flops = 2.0 * B * V * V * 32
    ach = flops / (ms * 1e-3) / 1e12
    return {"kernel": f"pk_feat_dist_topk (configs[1]: 32 x 1024 x 1024, fp32 top-{topk}, prep + main)", "bound": "mfma",
            "achieved": round(ach, 2), "peak": F32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / F32_MFMA_TFLOPS, 4),
            "ms_per_launch": round(ms, 4), "flops_per_launch": flops, "launches": launches}


def cpu_baseline(n_crops: int, n1: int, n2: int) -> dict:
    """The oracle (reference CPU path restated: numpy / torch-CPU) on the same synthetic
    inputs: crop formation + DPFM fwd+bwd + loss + naive IR + RMSprop, per crop."""
    from oracle import dpfm_oracle as O
    from oracle import dpfm_model_oracle as M
    from dpfm_amd.dataset.synthetic import make_frame, cad_points, lbo_operators
    # the box's CPU share, not the machine: OMP_NUM_THREADS is set to that share on the GPU
    # box (nproc / the affinity mask show every core of the host; oversubscribing them made
    # the torch-CPU model ~30x slower)
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(threads)
    model = M.DPFMNet()
    opt = torch.optim.RMSprop(model.parameters(), lr=5e-4)
    rng = np.random.default_rng(0)
    # BASELINE.md protocol: 2 untimed warm-up crops, then the sample in 5 equal parts; the
    # reported rate is the median of the 5 parts' rates
    parts = 5
    per = max(1, n_crops // parts)
    n_crops = per * parts
    marks = []
    t0 = time.perf_counter()
    for c in range(-2, n_crops):  # crops -2, -1: untimed warm-up (allocator, thread pool)
        if c >= 0 and c % per == 0:
            marks.append(time.perf_counter())
        cs = c % 10_000  # non-negative seeds for the warm-up crops
        fr = make_frame(10_000 + cs)
        pcd = O.dpt_2_pcld(fr.depth, 1000 / fr.depth_scale, fr.K, fr.mask == 255)
        pcd = O.remove_outliers(pcd)
        idx = O.farthest_point_sample(torch.Tensor(pcd).t(), ratio=n2 / pcd.shape[0], start=0, npoint=n2)
        pcd = pcd[idx.numpy()]
        align = O.transform(pcd, fr.R_m2c, fr.t_m2c, inv=True)
        cad = cad_points(fr, n1, cs)
        P = O.find_positives(cad, align, r=fr.diam_cad * 0.05)
        o12, o21 = O.get_overlap(n1, n2, P)
        cm, ce, cv = lbo_operators(n1, 64, 2 * cs)
        pm, pe, pv = lbo_operators(n2, 64, 2 * cs + 1)
        T = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float32))[None]  # noqa: E731
        batch = {"shape1": {"xyz": T(cad), "mass": T(cm), "evals": T(ce), "evecs": T(cv)},
                 "shape2": {"xyz": T(pcd), "mass": T(pm), "evals": T(pe), "evecs": T(pv)}}
        C, s12, s21, f1, f2, _, _ = model(batch)
        C_gt = M.C_from_sparse_P(torch.from_numpy(P), batch["shape1"]["evecs"][0, :, :30],
                                 batch["shape2"]["evecs"][0, :, :30])[None]
        sel = [torch.from_numpy(M.nce_selection(P.shape[0], 512, rng))]
        loss = M.dpfm_loss(C, C_gt, [torch.from_numpy(P)], sel, f1, f2, s12, s21, T(o12), T(o21))
        with torch.no_grad():
            p2p = O.naive_fmap2pointmap(C[0].detach(), batch["shape1"]["evecs"][0, :, :30],
                                        batch["shape2"]["evecs"][0, :, :30])
            O.compute_inlier_ratio(p2p.t(), T(cad)[0], T(align)[0], 0.1 * fr.diam_cad)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 5.0)
        opt.step()
        opt.zero_grad()
    marks.append(time.perf_counter())
    rates = sorted(per / (b - a) for a, b in zip(marks[:-1], marks[1:]))
    dt = marks[-1] - marks[0]
    import platform
    model_name = platform.processor()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model_name = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(rates[len(rates) // 2], 4), "unit": "crops/s (fwd+bwd incl. crop formation)",
            "cores": threads, "kind": "port",
            "sample": f"median of 5 x {per} crops after 2 warm-up crops, {n2} pts, CAD {n1}; oracle/ (numpy + "
                      f"torch-CPU fp32) on {model_name}",
            "rates": [round(r, 4) for r in rates], "seconds": round(dt, 2)}


def cpu_infer_baseline(n_crops: int, n1: int, n2: int, H: int) -> dict:
    """configs[1] inference on the host, per crop (scripts/eval.py:57-119 + test_RANSAC.py:
    397-419 restated by oracle/): crop formation, DPFMNet forward (torch-CPU fp32), the
    spatial-filtering solver (top-5 + three rigidity rounds), IR, the Open3D-shaped RANSAC
    (oracle/c oc_ransac_o3d, H hypotheses, C/OpenMP) and the ADD metric."""
    import ctypes
    from oracle import dpfm_oracle as O
    from oracle import dpfm_model_oracle as M
    from dpfm_amd.dataset.synthetic import make_frame, cad_points, lbo_operators
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    torch.set_num_threads(threads)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle.so"))
    P = ctypes.c_void_p
    lib.oc_ransac_o3d.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_uint64, ctypes.c_int64,
                                  ctypes.c_double, P, P]
    cp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    model = M.DPFMNet().eval()
    parts = 5  # BASELINE.md protocol: 2 warm-up crops, median of 5 equal parts
    per = max(1, n_crops // parts)
    n_crops = per * parts
    marks = []
    for c in range(-2, n_crops):  # crops -2, -1: untimed warm-up
        if c >= 0 and c % per == 0:
            marks.append(time.perf_counter())
        cs = c % 10_000
        fr = make_frame(20_000 + cs)
        pcd = O.dpt_2_pcld(fr.depth, 1000 / fr.depth_scale, fr.K, fr.mask == 255)
        pcd = O.remove_outliers(pcd)
        idx = O.farthest_point_sample(torch.Tensor(pcd).t(), ratio=n2 / pcd.shape[0], start=0, npoint=n2)
        pcd = pcd[idx.numpy()]
        align = O.transform(pcd, fr.R_m2c, fr.t_m2c, inv=True)
        cad = cad_points(fr, n1, cs)
        cm, ce, cv = lbo_operators(n1, 64, 2 * cs)
        pm, pe, pv = lbo_operators(n2, 64, 2 * cs + 1)
        T = lambda a: torch.from_numpy(np.asarray(a, dtype=np.float32))[None]  # noqa: E731
        batch = {"shape1": {"xyz": T(cad), "mass": T(cm), "evals": T(ce), "evecs": T(cv)},
                 "shape2": {"xyz": T(pcd), "mass": T(pm), "evals": T(pe), "evecs": T(pv)}}
        with torch.no_grad():
            C = model(batch)[0]
            corr = O.spacial_filtering_fmap2pointmap(C[0], batch["shape1"]["evecs"][0, :, :30],
                                                     batch["shape2"]["evecs"][0, :, :30], T(cad)[0], T(pcd)[0],
                                                     fr.diam_cad)
            O.compute_inlier_ratio(corr.t().long(), T(cad)[0], T(align)[0], 0.1 * fr.diam_cad)
        cor = np.ascontiguousarray(corr.t().numpy().astype(np.int32))
        Tm, st = np.zeros(16), np.zeros(3)
        cad64, pc64 = np.ascontiguousarray(cad, dtype=np.float64), np.ascontiguousarray(pcd, dtype=np.float64)
        if cor.shape[0] >= 4:
            lib.oc_ransac_o3d(cp(cad64), n1, cp(pc64), cp(cor), cor.shape[0], None, 0, H, 0.05, cp(Tm), cp(st))
        Tgt = np.eye(4)
        Tgt[:3, :3], Tgt[:3, 3] = fr.R_m2c, fr.t_m2c
        O.add(Tm.reshape(4, 4), Tgt, cad, fr.diam_cad)
    marks.append(time.perf_counter())
    rates = sorted(per / (b - a) for a, b in zip(marks[:-1], marks[1:]))
    dt = marks[-1] - marks[0]
    return {"value": round(rates[len(rates) // 2], 4), "unit": "crops/s (inference incl. crop formation and RANSAC)",
            "cores": threads, "kind": "port",
            "sample": f"median of 5 x {per} crops after 2 warm-up crops, {n2} pts, CAD {n1}, RANSAC {H} hypotheses; "
                      "oracle/ (numpy + torch-CPU fp32, C/OpenMP RANSAC)",
            "rates": [round(r, 4) for r in rates], "seconds": round(dt, 2)}


def cpu_pose_check(model, fb, op, crops, out: dict, n_sample: int, H: int, seed: int) -> dict:
    """The metric's "pose err vs ref": the device pose path (InferStep: DPFMNet forward ->
    top-5 -> rigidity filter -> RANSAC, already run, `out`) against the reference CPU path
    restated by oracle/ on the SAME crops and weights, for a bounded sample of crops:
      end_to_end   torch-CPU fp32 DPFMNet -> spacial_filtering_fmap2pointmap -> C RANSAC (the
                   same hash-drawn hypotheses) -> T_ref, compared with the device T;
      same_corr    the C RANSAC on the device's own survivors (isolates the pose stage).
    ADD (test_RANSAC.py:162-173) of both poses vs T_gt. North-star tolerance: 1e-4."""
    import ctypes
    from oracle import dpfm_oracle as O
    from oracle import dpfm_model_oracle as M
    from dpfm_amd.pipeline import model_batch
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle.so"))
    P = ctypes.c_void_p
    lib.oc_ransac.argtypes = [P, P, P, ctypes.c_int, P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, P, P]
    cp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    ref = M.DPFMNet().eval()
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    mb = model_batch(op, crops)
    B = int(crops.off.numel() - 1)
    n = min(n_sample, B)
    keys = ("xyz", "mass", "evals", "evecs")
    cpu = {k: {kk: vv[:n].cpu() for kk, vv in v.items() if kk in keys} for k, v in mb.items()}
    T_dev = out["T"].cpu().numpy()
    p_pred, ncorr = out["p_pred"].cpu().numpy(), out["n_corr"].cpu().numpy()
    cad64, cad_off = fb.cad64.cpu().numpy(), fb.cad_off.cpu().numpy()
    pc64, off = crops.pc64.cpu().numpy(), crops.off.cpu().numpy()
    t0 = time.perf_counter()
    with torch.no_grad():
        C_ref = ref(cpu)[0]
    e2e, same, within, add_dev, add_ref = [], [], 0, [], []
    for b in range(n):
        cad_b = np.ascontiguousarray(cad64[cad_off[b]:cad_off[b + 1]])
        pc_b = np.ascontiguousarray(pc64[off[b]:off[b + 1]])
        ex, ey = cpu["shape1"]["evecs"][b, :, :30], cpu["shape2"]["evecs"][b, :, :30]
        with torch.no_grad():
            corr = O.spacial_filtering_fmap2pointmap(C_ref[b], ex, ey, cpu["shape1"]["xyz"][b], cpu["shape2"]["xyz"][b],
                                                     fb.diam[b])
        T_ref = np.zeros(16)
        st = np.zeros(3)
        cor = np.ascontiguousarray(corr.t().numpy().astype(np.int32))
        lib.oc_ransac(cp(cad_b), cp(pc_b), cp(cor), int(cor.shape[0]), None, seed, H, 0.05, cp(T_ref), cp(st))
        T_s = np.zeros(16)
        cs = np.ascontiguousarray(p_pred[b, :ncorr[b]].astype(np.int32))
        lib.oc_ransac(cp(cad_b), cp(pc_b), cp(cs), int(ncorr[b]), None, seed, H, 0.05, cp(T_s), cp(st))
        d = float(np.abs(T_dev[b] - T_ref.reshape(4, 4)).max())
        e2e.append(d)
        within += d <= 1e-4
        same.append(float(np.abs(T_dev[b] - T_s.reshape(4, 4)).max()))
        T_gt = np.eye(4)
        T_gt[:3, :3] = fb.R[b].cpu().numpy().reshape(3, 3)
        T_gt[:3, 3] = fb.t[b].cpu().numpy()
        add_dev.append(O.add(T_dev[b], T_gt, cad_b, fb.diam[b])[0])
        add_ref.append(O.add(T_ref.reshape(4, 4), T_gt, cad_b, fb.diam[b])[0])
    return {"crops": n, "hypotheses": H, "tolerance": 1e-4,
            "end_to_end_max_abs_dT": round(max(e2e), 12), "end_to_end_crops_within_tol": int(within),
            "same_corr_max_abs_dT": round(max(same), 15),
            "mean_add_device": round(float(np.mean(add_dev)), 6), "mean_add_ref": round(float(np.mean(add_ref)), 6),
            "seconds": round(time.perf_counter() - t0, 2),
            "note": "device InferStep vs oracle/ (torch-CPU fp32 model, spacial filtering, C RANSAC on the same "
                    "hypothesis draws) on the same crops and weights; same_corr runs the oracle RANSAC on the "
                    "device's survivors; ADD in cm vs the synthetic T_gt (random-init weights: ADD is large)"}


def pose_real_check(dev, H: int = 1024, seed: int = 7, inlier_frac: float = 0.4, noise_cm: float = 0.005) -> dict:
    """The metric's "pose err vs ref" on correspondences with real inliers: the 7 published
    crops of tests/golden/real_crops.npz (the reference's own camera-frame crops pc_i.ply,
    their decimated CADs and full-precision T_gt). Per crop the target cloud is the real crop
    plus planted points: a fraction `inlier_frac` of the correspondences are CAD vertices i
    paired with T_gt CAD[i] + N(0, noise_cm) (inside test_RANSAC.py's 0.05 cm threshold), the
    rest (>= 60 %) pair every real crop point with a random CAD vertex (outliers). Device
    pk_ransac (batched over the 7 crops) vs the oracle's C RANSAC (Open3D semantics restated,
    oracle/c/oracle.c) on the same hash-drawn hypotheses: fitness, rotation / translation error
    vs T_gt and max |dT| between the two (north-star tolerance 1e-4)."""
    import ctypes
    from dpfm_amd import ops
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "liboracle.so"))
    P = ctypes.c_void_p
    lib.oc_ransac.argtypes = [P, P, P, ctypes.c_int, P, ctypes.c_uint64, ctypes.c_int64, ctypes.c_double, P, P]
    cp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    G = np.load(os.path.join(ROOT, "tests", "golden", "real_crops.npz"))
    rng = np.random.default_rng(seed)
    cads, pcs, cors, Tg = [], [], [], []
    for k in range(int(G["n"])):
        cad = np.ascontiguousarray(G[f"cad_{int(G[f'{k}_obj_id'])}"], dtype=np.float64)
        pc = np.asarray(G[f"{k}_pc"], dtype=np.float64)
        T = np.asarray(G[f"{k}_T_gt"], dtype=np.float64)
        n_out = pc.shape[0]
        n_in = int(round(n_out * inlier_frac / (1.0 - inlier_frac)))
        ci = rng.integers(0, cad.shape[0], n_in)
        planted = cad[ci] @ T[:3, :3].T + T[:3, 3] + rng.normal(size=(n_in, 3)) * noise_cm
        tgt = np.ascontiguousarray(np.concatenate([planted, pc]))
        cor = np.concatenate([np.stack([ci, np.arange(n_in)], 1),
                              np.stack([rng.integers(0, cad.shape[0], n_out), n_in + np.arange(n_out)], 1)])
        cor = np.ascontiguousarray(cor[rng.permutation(cor.shape[0])].astype(np.int32))
        cads.append(cad), pcs.append(tgt), cors.append(cor), Tg.append(T)
    off = lambda a: torch.tensor(np.concatenate([[0], np.cumsum([x.shape[0] for x in a])]), dtype=torch.int64,  # noqa
                                 device=dev)
    Td, st = ops.ransac(torch.from_numpy(np.concatenate(cads)).to(dev), off(cads),
                        torch.from_numpy(np.concatenate(pcs)).to(dev), off(pcs),
                        torch.from_numpy(np.concatenate(cors)).to(dev), off(cors), H, seed=seed, max_dist=0.05)
    Td, st = Td.cpu().numpy(), st.cpu().numpy()
    dT, fit, rot, tra, fit_ref = [], [], [], [], []
    for k in range(len(cads)):
        T_ref, s_ref = np.zeros(16), np.zeros(3)
        lib.oc_ransac(cp(cads[k]), cp(pcs[k]), cp(cors[k]), int(cors[k].shape[0]), None, seed, H, 0.05, cp(T_ref),
                      cp(s_ref))
        dT.append(float(np.abs(Td[k] - T_ref.reshape(4, 4)).max()))
        fit.append(float(st[k, 0]))
        fit_ref.append(float(s_ref[0]))
        Rr = Td[k][:3, :3] @ Tg[k][:3, :3].T
        rot.append(float(np.degrees(np.arccos(np.clip((np.trace(Rr) - 1) / 2, -1, 1)))))
        tra.append(float(np.linalg.norm(Td[k][:3, 3] - Tg[k][:3, 3])))
    return {"crops": len(cads), "hypotheses": H, "tolerance": 1e-4, "max_abs_dT_vs_oracle": round(max(dT), 15),
            "crops_within_tol": int(sum(d <= 1e-4 for d in dT)), "fitness_min": round(min(fit), 4),
            "fitness_mean": round(float(np.mean(fit)), 4), "fitness_equal_to_oracle": fit == fit_ref,
            "rot_err_deg_max": round(max(rot), 5), "trans_err_cm_max": round(max(tra), 5),
            "inlier_fraction_planted": inlier_frac,
            "note": "the reference's 7 published real crops (tests/golden/real_crops.npz) + planted inliers "
                    f"(N(0, {noise_cm} cm) around T_gt CAD[i]); outliers: every real crop point paired with a "
                    "random CAD vertex; device pk_ransac vs the C oracle on the same hypothesis draws"}


TRAIN_METRIC = "RGB-D crops/sec (fwd+bwd), 1024 pts, at 1/2/4/8 MI355X; pose err vs ref"
INFER_METRIC = ("RGB-D crops/sec (inference: crop formation + DPFM fwd + spatial-filter solver + IR + "
                "RANSAC 1024 hyp + pose metrics)")
CORR_METRIC = "4096-pt dense correspondence solves/sec (4096^2 feature distance + 1024-hypothesis RANSAC)"
OPS_METRIC = "crop spectral operators/sec (kNN-30 fans + cotan Laplacian + mass + 64 eigenpairs)"
TEASER_METRIC = "TEASER++ solves/sec (pairwise-consistency graph + max clique + GNC-TLS + adaptive voting)"
ICP_METRIC = "ICP refinements/sec (point-to-point after RANSAC, ~5000-vertex CAD, threshold 0.2 cm, <= 2000 iterations)"
CROP_FAMS = {"pk_backproject", "pk_sor", "pk_fps_npoint", "pk_fps", "pk_gather_transform", "pk_gather_transform_pad",
             "pk_collate_pad",
             "pk_ball_query_mask", "pk_ball_query_pairs", "pk_sample_rgb", "pk_erode_mask"}


def launcher_cmd(argv, env) -> list | None:
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launcher: the command that
    starts N ranks (one process per GPU) as a CHILD process, or None when this process is
    already a rank (WORLD_SIZE set) or N == 1. The parent never touches the GPU; it waits for
    the child and exits with its code (no exec from a process that initialised HIP)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    known, _ = ap.parse_known_args(argv)
    if "WORLD_SIZE" in env or known.gpus <= 1:
        return None
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={known.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def setup_dist(gpus: int = 0):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if gpus and world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}; launch with --nproc-per-node {gpus}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knob: PK_BENCH_BACKEND=gloo with more ranks than GPUs shares the cards
    # round-robin (the driver's multi-GPU runs use RCCL, one rank per GPU)
    backend = os.environ.get("PK_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    return world, rank, dev


POSE_CHECK = {}  # mode -> the post-timing pose-vs-reference check (cpu_baseline leg)


def ragged_setup(B: int, n1: int, rank: int, dev):
    """The reference's real sizes: frames whose masks give ~200-2000-point crops under
    the sample policy (CropFormation(npoint=0), padded to the policy maximum 2000 so the step is
    graph-capturable), CADs of ~n1 vertices, and the cached-operator stand-ins of those sizes
    (operators_for reads the crop sizes once, at setup: the reference computes them offline)."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.dataset.synthetic import ragged_frames
    from dpfm_amd.pipeline import frame_batch, operators_for
    frames = ragged_frames(B, 1000 * rank + 77, n1=n1)
    fb = frame_batch(frames, dev)
    crops_of = CropFormation(npoint=0, seed=rank, pad="fixed", base=rank * B)
    c0 = crops_of(fb)
    counts = c0.n2.cpu().tolist()
    op = operators_for([f["cad"] for f in frames], counts, fb.diam, 1000 * rank, dev, ld2=c0.ld)
    cads = [len(f["cad"]) for f in frames]
    sizes = {"crop_min": int(min(counts)), "crop_max": int(max(counts)), "crop_mean": round(float(np.mean(counts)), 1),
             "cad_min": min(cads), "cad_max": max(cads), "cad_mean": round(float(np.mean(cads)), 1)}
    return fb, op, crops_of, sizes


def train_workload(B: int, N: int, world: int) -> str:
    """The training line's workload name: which BASELINE.json config the (per-rank batch, world)
    pair IS, with the true global batch stated."""
    shape = f"synthetic 640x480 RGB-D crops, {N} pts, training step fwd+bwd"
    if world == 1:
        return f"configs[1] shape: B={B} {shape} on 1 GPU (global batch {B})"
    if world == 2 and B * world == 32 and N == 1024:
        return f"configs[2]: global batch 32 = 2 ranks x B=16, {shape}, DDP with RCCL gradient all-reduce"
    return (f"configs[1] shape per GPU, weak scaling: global batch {B * world} = {world} ranks x B={B}, {shape}, "
            f"DDP with RCCL gradient all-reduce (configs[2] itself: --gpus 2 --global-batch 32)")


def apply_global_batch(args, world: int) -> None:
    """--global-batch G: G crops over all ranks (G / world per rank; must divide)."""
    if args.global_batch is None:
        return
    if args.global_batch % world:
        raise SystemExit(f"bench.py: --global-batch {args.global_batch} is not divisible by {world} ranks")
    args.batch = args.global_batch // world


def build_train(args, dev, rank, world):
    """configs[1] shape (configs[2] semantics for N > 1): one training step per iteration."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedTrainStep, PipelinedTrainer, TrainStep, make_frame_batch
    B, N = args.batch, args.points
    torch.manual_seed(1234)  # identical initial weights on every rank (DDP broadcast semantics)
    model = DPFMNet().to(dev)
    if args.ragged:
        fb, op, crops_of, sizes = ragged_setup(B, args.cad_points, rank, dev)
    else:
        fb, op = make_frame_batch(B, N, N, seed=1000 * rank, device=dev)
        crops_of = CropFormation(n1=N, npoint=N, seed=rank)
    step = TrainStep(model, seed=rank, capturable=not args.eager)
    if args.eager:
        one_step = lambda: step(op, crops_of(fb))  # noqa: E731
    elif args.train_only:  # diagnostic: the training stream alone, on one fixed crop batch
        fixed = crops_of(fb)
        one_step = GraphedTrainStep(lambda _fb: fixed, step, fb, op, warmup=3)
    elif args.no_overlap:  # warm-up + capture (untimed), then every step is a graph replay
        one_step = GraphedTrainStep(crops_of, step, fb, op, warmup=3)
    else:  # same, with crop formation of the next batch on a second stream
        one_step = PipelinedTrainer(crops_of, step, fb, op, warmup=3, main_priority=args.main_priority,
                                        side_cus=args.side_cus, side_after=args.side_after,
                                        cgt_side=bool(args.ragged) if args.cgt_side is None else bool(args.cgt_side),
                                        defer_ir=not args.ir_main)
    config = {"workload": train_workload(B, N, world),
              "execution": "eager" if args.eager else ("hip-graph, training only (diagnostic)" if args.train_only else
                                                       "hip-graph" if args.no_overlap else
                                                       "hip-graph, crop formation overlapped" +
                                                       (", pose stage of the previous batch overlapped"
                                                        if args.infer_stages == 3 else "")),
              "global_batch": B * world, "points_per_crop": N, "cad_points": N,
              "precision": "model fp32 (f32 MFMA); crop geometry / C_gt normal equations fp64",
              "parallelism": f"dp{world}"}
    if args.ragged:
        config.update(workload=f"reference sizes: B={B} synthetic 640x480 RGB-D frames/GPU, ragged crops "
                               f"{sizes['crop_min']}-{sizes['crop_max']} pts (sample policy, collate padding to 2000), "
                               f"CADs {sizes['cad_min']}-{sizes['cad_max']} vertices, training step fwd+bwd",
                      points_per_crop=sizes["crop_mean"], cad_points=sizes["cad_mean"])
    probe = lambda: step(op, crops_of(fb))  # noqa: E731

    def pose_check(n_sample):  # the metric's "pose err vs ref" on the trained weights (after timing)
        from dpfm_amd.pipeline import InferStep
        crops = crops_of(fb)
        out = InferStep(model, hypotheses=1024, seed=5)(fb, op, crops)
        torch.cuda.synchronize()
        return cpu_pose_check(model, fb, op, crops, out, n_sample, 1024, 5)
    POSE_CHECK["fn"] = pose_check
    return one_step, probe, TRAIN_METRIC, B, config


def build_infer(args, dev, rank, world):
    """configs[1] (B = 32 x 1024 pts, 1 GPU) / configs[3] (--points 2048; each rank infers its
    own shard of the batch, no collective on the data path): one inference pass per iteration."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedInfer, InferStep, PipelinedInfer, make_frame_batch
    B, N = args.batch, args.points
    torch.manual_seed(1234)
    model = DPFMNet().to(dev).eval()
    if args.ragged:
        fb, op, crops_of, sizes = ragged_setup(B, args.cad_points, rank, dev)
    else:
        fb, op = make_frame_batch(B, N, N, seed=1000 * rank, device=dev)
        crops_of = CropFormation(n1=N, npoint=N, seed=0, base=rank * B)
    infer = InferStep(model, hypotheses=args.hypotheses, seed=0, icp_evaluations=args.icp_evals)
    if args.eager:
        one_step = lambda: infer(fb, op, crops_of(fb))  # noqa: E731
    elif args.no_overlap:
        one_step = GraphedInfer(crops_of, infer, fb, op)
    else:  # crop formation of the next batch on a second stream, as in training
        one_step = PipelinedInfer(crops_of, infer, fb, op, stages=args.infer_stages)
    name = "configs[3] shard" if N == 2048 else "configs[1]"
    config = {"workload": f"{name}: B={B} synthetic 640x480 RGB-D crops/GPU, {N} pts, inference (eval.py + "
                          f"test_RANSAC.py: top-5 + 3-round rigidity filter + IR + RANSAC {args.hypotheses} "
                          "hypotheses + ADD metrics" + (f" + ICP to the crop ({args.icp_evals} evaluations)"
                                                         if args.icp_evals else "") +
                          "), batch-sharded across ranks (weak scaling)",
              "execution": "eager" if args.eager else ("hip-graph" if args.no_overlap else
                                                       "hip-graph, crop formation overlapped" +
                                                       (", pose stage of the previous batch overlapped"
                                                        if args.infer_stages == 3 else "")),
              "global_batch": B * world, "points_per_crop": N, "cad_points": N, "hypotheses": args.hypotheses,
              "precision": "model fp32 (f32 MFMA); crop geometry / RANSAC fp64", "parallelism": f"shard{world}"}
    if args.ragged:
        config.update(workload=f"reference sizes: B={B} synthetic 640x480 RGB-D frames/GPU, ragged crops "
                               f"{sizes['crop_min']}-{sizes['crop_max']} pts (collate padding to 2000), CADs "
                               f"{sizes['cad_min']}-{sizes['cad_max']} vertices, inference + RANSAC "
                               f"{args.hypotheses} hypotheses", points_per_crop=sizes["crop_mean"],
                      cad_points=sizes["cad_mean"])
    probe = lambda: infer(fb, op, crops_of(fb))  # noqa: E731
    return one_step, probe, INFER_METRIC, B, config


def build_corr(args, dev, rank, world):
    """configs[4]: one 4096-point crop vs a 4096-vertex CAD: the naive solver's feature
    distance (naive.py:20-33, 4096 x 4096 x 30) and RANSAC with 1024 hypotheses over the
    4096 point-map correspondences (test_RANSAC.py:288-310)."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import lbo_operators, random_rotation
    V, H = 4096, args.hypotheses
    rng = np.random.default_rng(4096 + rank)
    ex = torch.from_numpy(lbo_operators(V, 64, 1)[2])[None].to(dev)
    ey = torch.from_numpy(lbo_operators(V, 64, 2)[2])[None].to(dev)
    C = (torch.eye(30) + 0.1 * torch.randn(30, 30, generator=torch.Generator().manual_seed(3)))[None].to(dev)
    cad = rng.normal(size=(V, 3)) * 6
    R = random_rotation(rng)
    pc = (cad[rng.permutation(V)] + rng.normal(size=(V, 3)) * 0.02) @ R.T + np.array([2.0, -1.0, 90.0])
    cad_t, pc_t = torch.from_numpy(cad).to(dev), torch.from_numpy(pc).to(dev)
    off = torch.tensor([0, V], dtype=torch.int64, device=dev)
    n = torch.full((1,), V, dtype=torch.int32, device=dev)
    ar = torch.arange(V, dtype=torch.int32, device=dev)
    bf16 = args.fd_precision != "fp32"

    st_idx = torch.zeros((1,), dtype=torch.int32, device=dev)  # persistent: no per-call host check

    def solve():
        idx, _ = ops.feat_dist_topk(ex, C, ey, n, n, 1, precision=args.fd_precision)
        corres = torch.stack([idx[0, :, 0].to(torch.int32), ar], 1)
        return {"T": ops.ransac(cad_t, off, pc_t, off, corres, off, H, seed=0, nmax=V, status=st_idx)[0],
                "index_status": st_idx}

    one_step = solve
    if not args.eager:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                solve()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = solve()

        def one_step():
            g.replay()
            return out
    config = {"workload": f"configs[4]: one crop, V1 = V2 = {V}: feature distance {V}x{V}x30 "
                          f"({args.fd_precision} MFMA, K padded to 32) + argmin + RANSAC {H} hypotheses "
                          f"over n = {V} correspondences", "execution": "eager" if args.eager else "hip-graph",
              "global_batch": world, "points_per_crop": V, "cad_points": V, "hypotheses": H,
              "precision": (f"{args.fd_precision} cross term / f32 norms and accumulate" if bf16 else "fp32")
              + " distance; fp64 RANSAC",
              "parallelism": f"replicas{world}"}
    return one_step, solve, CORR_METRIC, 1, config


def icp_workload(B: int, rank: int, target: str):
    """(f4) workload per rank: B CADs of 5000 surface points (ellipsoids, semi-axes 4-8 cm, the
    reference's decimated CAD size), a random T_gt per crop, init = T_gt perturbed by 3 degrees
    and ~0.1 cm (a RANSAC-quality start); target = the CAD under T_gt (test_RANSAC.py:426-436)
    or a 2000-point noisy partial view of it (the observed-crop variant)."""
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(777 + rank)
    srcs, tgts, T0s = [], [], []
    for b in range(B):
        ax = rng.uniform(4, 8, size=3)
        u = rng.normal(size=(5000, 3))
        src = u / np.linalg.norm(u, axis=1, keepdims=True) * ax
        R = random_rotation(rng)
        t = rng.normal(size=3) * 10 + np.array([0, 0, 90.0])
        Tg = np.eye(4)
        Tg[:3, :3], Tg[:3, 3] = R, t
        tgt = src @ R.T + t
        if target == "crop":
            vis = (src @ R.T)[:, 2] < 0  # the half facing the camera
            idx = np.flatnonzero(vis)[:2000]
            tgt = tgt[idx] + rng.normal(size=(idx.size, 3)) * 0.02
        a = np.deg2rad(3.0)
        k = rng.normal(size=3)
        k /= np.linalg.norm(k)
        K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
        D = np.eye(4)
        D[:3, :3] = np.eye(3) + np.sin(a) * K + (1 - np.cos(a)) * K @ K
        D[:3, 3] = t - D[:3, :3] @ t + rng.normal(size=3) * 0.1
        srcs.append(src)
        tgts.append(np.ascontiguousarray(tgt))
        T0s.append(D @ Tg)
    return srcs, tgts, T0s


RANSAC_REF_METRIC = ("reference pose-stage solves/sec (test_RANSAC.py:288-310: 4x10^6 RANSAC hypotheses per "
                     "crop over ~760 correspondences, ~5000-vertex CAD)")


def build_ransac_ref(args, dev, rank, world):
    """The reference's own pose workload (test_RANSAC.py:308, call at :400): per crop 4 x 10^6
    hypotheses (RANSACConvergenceCriteria(4000000, 80000): confidence clamps to 1, so every
    hypothesis runs) over the spatially filtered correspondences (n ~ 450-770 on its real crops)
    with a ~5000-vertex CAD. Synthetic: n = 760 correspondences, 40 % inliers, B = --batch crops
    per step (default 1 here: one crop's solve per step)."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.synthetic import random_rotation
    H = args.hypotheses if args.hypotheses != 1024 else 4_000_000
    B, V1, n = max(1, args.ransac_crops), args.cad_points, 760
    rng = np.random.default_rng(7000 + rank)
    cads, pcs, cors = [], [], []
    for b in range(B):
        cad = rng.normal(size=(V1, 3)) * 6
        R = random_rotation(rng)
        gen = rng.integers(0, V1, n)
        pc = (cad[gen] + rng.normal(size=(n, 3)) * 0.01) @ R.T + np.array([2.0, -1.0, 90.0])
        src = rng.integers(0, V1, n)
        good = rng.random(n) < 0.4
        src[good] = gen[good]
        cads.append(cad)
        pcs.append(pc)
        cors.append(np.stack([src, np.arange(n)], 1))
    cad_t = torch.from_numpy(np.concatenate(cads)).to(dev)
    pc_t = torch.from_numpy(np.concatenate(pcs)).to(dev)
    cad_off = ops.packed_offsets([V1] * B, dev)
    pc_off = ops.packed_offsets([n] * B, dev)
    corres = torch.from_numpy(np.concatenate(cors).astype(np.int32)).to(dev)
    cor_off = ops.packed_offsets([n] * B, dev)

    st_idx = torch.zeros((B,), dtype=torch.int32, device=dev)  # persistent: no per-call host check

    def solve():
        T, st = ops.ransac(cad_t, cad_off, pc_t, pc_off, corres, cor_off, H, seed=0, nmax=n, status=st_idx)
        return {"T": T, "stats": st, "index_status": st_idx}

    one_step = solve
    if not args.eager:
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            solve()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = solve()

        def one_step():
            g.replay()
            return out
    config = {"workload": f"reference pose stage: {B} crop(s) x {H} RANSAC hypotheses x {n} correspondences "
                          f"(40 % inliers), {V1}-vertex CAD, fp64 Umeyama/Horn fit + scoring",
              "execution": "eager" if args.eager else "hip-graph", "global_batch": B * world, "hypotheses": H,
              "correspondences": n, "cad_points": V1, "precision": "fp64", "parallelism": f"shard{world}"}
    return one_step, solve, RANSAC_REF_METRIC, B, config


def build_icp(args, dev, rank, world):
    """(f4): batched ICP of B crops per rank (test_RANSAC.py:436-446), crops sharded across
    ranks with no collective. One step = the whole refinement of the batch, including the
    host's convergence polls (one 4-byte read per 8 evaluations)."""
    from dpfm_amd import ops
    B = args.batch
    srcs, tgts, T0s = icp_workload(B, rank, args.icp_target)
    cat = lambda a: torch.from_numpy(np.ascontiguousarray(np.concatenate(a, 0))).to(dev)  # noqa: E731
    offs = lambda a: torch.from_numpy(np.concatenate([[0], np.cumsum([x.shape[0] for x in a])])).to(dev)  # noqa
    s, so, t, to = cat(srcs), offs(srcs), cat(tgts), offs(tgts)
    T0 = torch.from_numpy(np.stack(T0s)).to(dev)
    nsm, ntm = max(x.shape[0] for x in srcs), max(x.shape[0] for x in tgts)
    state = {}

    def one_step():
        T, st = ops.icp(s, so, t, to, T0, 0.2, 2000, nsrc_max=nsm, ntgt_max=ntm)
        state["stats"] = st
        return {"T": T, "stats": st}
    config = {"workload": f"(f4) ICP: B={B} crops/GPU, source = 5000-point CAD, target = "
                          + ("the CAD under T_gt (the reference's)" if args.icp_target == "gt_cad" else
                             "a 2000-point noisy partial view (observed-crop variant)")
                          + ", threshold 0.2 cm, max_iteration 2000, relative fitness / rmse 1e-6, init = T_gt "
                            "perturbed by 3 deg", "execution": "eager, host polls convergence every 8 evaluations",
              "global_batch": B * world, "points_per_crop": 5000, "precision": "fp64",
              "parallelism": f"shard{world}"}
    return one_step, one_step, ICP_METRIC, B, config


def ops_workload(B: int, n: int, rank: int):
    """(f1) per rank: B crop-like point clouds of n points: the camera-facing half of an ellipsoid
    (semi-axes 4-8 cm) with 0.02 cm noise — the shape of an eroded, outlier-filtered depth crop."""
    rng = np.random.default_rng(99 + rank)
    out = []
    for _ in range(B):
        ax = rng.uniform(4, 8, size=3)
        u = rng.normal(size=(4 * n, 3))
        u = u[u[:, 2] < 0][:n]
        out.append(u / np.linalg.norm(u, axis=1, keepdims=True) * ax + rng.normal(size=(n, 3)) * 0.02)
    return out


def build_operators(args, dev, rank, world):
    """(f1): get_operators for B crops per rank (the reference's pc_LBO cache fill,
    dataset/object.py:246), no collective."""
    from dpfm_amd import geometry
    B, n = args.batch, args.op_points
    shapes = ops_workload(B, n, rank)
    state = {}

    def one_step():
        op = geometry.get_operators(shapes, k_eig=64, device=dev)
        state["it"] = op.iterations
        return {"iterations": op.iterations, "residual": float(op.residual.max())}
    config = {"workload": f"(f1) spectral operators: B={B} crop point clouds/GPU x {n} points, kNN 30, local Delaunay "
                          "fans, cotan Laplacian / 3, lumped mass, 64 smallest eigenpairs of L v = lambda M v "
                          "(Chebyshev-filtered subspace iteration, m = 128, degree 24, tol 1e-8)",
              "execution": "eager; host Rayleigh-Ritz per iteration", "global_batch": B * world, "points_per_crop": n,
              "precision": "fp64", "parallelism": f"shard{world}"}
    return one_step, one_step, OPS_METRIC, B, config


def cpu_ops_baseline(n_crops: int, n: int) -> dict:
    """oracle/operators_oracle.py on the host: numpy kNN, scipy (Qhull) Delaunay per neighbourhood,
    the cotan assembly and scipy eigsh(sigma = eps) — the same steps as compute_operators."""
    from oracle import operators_oracle as OO
    shapes = ops_workload(n_crops, n, 0)
    t0 = time.perf_counter()
    for s in shapes:
        idx, _ = OO.knn(s, 30)
        L, M = OO.cotan_laplacian(s, OO.local_triangles(s, idx), scale=1.0 / 3.0, denom_eps=0.0)
        OO.eigsh_operators(L, M, 64)
    dt = time.perf_counter() - t0
    return {"value": round(n_crops / dt, 4), "unit": "operator sets/s", "cores": 1, "kind": "port",
            "sample": f"{n_crops} crops x {n} points: numpy kNN, per-point scipy Delaunay fans (Python loop), "
                      "cotan assembly (Python loop), scipy eigsh shift-invert",
            "seconds": round(dt, 3)}


def teaser_workload(B: int, n: int, rank: int):
    """(f2) per rank: B crops of n correspondences (CAD points in cm, ~10 cm objects), 40 %
    planted inliers under a random pose with 0.01 cm noise, the rest random points around the
    object (the spatial-filter output the reference hands TEASER++, test_teaser.py:366-425)."""
    from dpfm_amd.dataset.synthetic import random_rotation
    rng = np.random.default_rng(4242 + rank)
    A, Bm = [], []
    for _ in range(B):
        R = random_rotation(rng)
        t = rng.normal(size=3) * 10 + np.array([0, 0, 90.0])
        a = rng.normal(size=(n, 3)) * 5
        b = a @ R.T + t + rng.normal(size=(n, 3)) * 0.01
        out = rng.random(n) >= 0.4
        b[out] = rng.normal(size=(int(out.sum()), 3)) * 5 + t
        A.append(a)
        Bm.append(b)
    return A, Bm


def build_teaser(args, dev, rank, world):
    """(f2): TEASER++ for B crops per rank, no collective. One step = device graph + one
    download of the bitsets + the host clique / GNC-TLS / voting on 16 threads."""
    from dpfm_amd import ops
    B, n = args.batch, args.teaser_n
    A, Bm = teaser_workload(B, n, rank)
    a = torch.from_numpy(np.concatenate(A)).to(dev)
    b = torch.from_numpy(np.concatenate(Bm)).to(dev)
    off = torch.arange(0, (B + 1) * n, n, dtype=torch.int64, device=dev)

    def one_step():
        T, clique, size, info = ops.teaser(a, b, off, n, threads=16)
        return {"info": info, "size": size}
    config = {"workload": f"(f2) TEASER++: B={B} crops/GPU x {n} correspondences (40 % inliers), noise_bound 0.05, "
                          "cbar2 1, no scaling, GNC-TLS 1.4 / 100 / 1e-12, max clique (k-core heuristic 0.5)",
              "execution": "eager: device graph, host solve on 16 threads", "global_batch": B * world,
              "correspondences": n, "precision": "fp64", "parallelism": f"shard{world}"}
    return one_step, one_step, TEASER_METRIC, B, config


def cpu_teaser_baseline(n_crops: int, n: int) -> dict:
    """The same solve with the consistency graph built on the host (numpy, the oracle's
    vectorized restatement) instead of the device; the clique / GNC / voting stage is the same
    native host code on 16 threads."""
    from oracle import dpfm_oracle as O
    from dpfm_amd import _lib, ops
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    A, Bm = teaser_workload(n_crops, n, 0)
    W = (n + 63) // 64
    p = _lib.TeaserParams(0.05, 1.0, 1.4, 1e-12, 0.5, 100, 0, 2_000_000)
    t0 = time.perf_counter()
    adj = np.zeros((n_crops, n, W), np.uint64)
    deg = np.zeros((n_crops, n), np.int32)
    for k in range(n_crops):
        g = O.teaser_graph(A[k], Bm[k], 0.1)
        full = np.zeros((n, W * 64), bool)
        full[:, :n] = g
        adj[k] = np.packbits(full, axis=1, bitorder="little").view(np.uint64)
        deg[k] = g.sum(1)
    off = np.arange(0, (n_crops + 1) * n, n, dtype=np.int64)
    ops.teaser_solve_host(np.concatenate(A), np.concatenate(Bm), off, n, adj, deg, p, threads)
    dt = time.perf_counter() - t0
    return {"value": round(n_crops / dt, 4), "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{n_crops} crops x {n} correspondences: numpy consistency graph + the native host solve",
            "seconds": round(dt, 3)}


def cpu_icp_baseline(n_crops: int, target: str) -> dict:
    """The same ICP loop on the host the way Open3D runs it: a KD-tree nearest-neighbour query
    per evaluation (scipy cKDTree, C++, `workers` threads, distance_upper_bound = threshold)
    and an SVD Umeyama, on the first n_crops crops of the same workload."""
    from scipy.spatial import cKDTree
    from oracle import dpfm_oracle as O
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    srcs, tgts, T0s = icp_workload(n_crops, 0, target)
    iters = 0
    t0 = time.perf_counter()
    for src, tgt, T in zip(srcs, tgts, T0s):
        tree = cKDTree(tgt)

        def evaluate(T):
            p = src @ T[:3, :3].T + T[:3, 3]
            d, j = tree.query(p, k=1, distance_upper_bound=0.2, workers=threads)
            ok = np.isfinite(d) & (d < 0.2)
            n = int(ok.sum())
            return p[ok], tgt[j[ok]], (n / len(p) if n else 0.0), (float(np.sqrt((d[ok] ** 2).sum() / n)) if n else 0.0)
        P, Q, fit, rmse = evaluate(T)
        for it in range(2000):
            T = (O.umeyama(P.T, Q.T) if len(P) else np.eye(4)) @ T
            pf, pr = fit, rmse
            P, Q, fit, rmse = evaluate(T)
            iters += 1
            if abs(pf - fit) < 1e-6 and abs(pr - rmse) < 1e-6:
                break
    dt = time.perf_counter() - t0
    return {"value": round(n_crops / dt, 4), "unit": "refinements/s", "cores": threads, "kind": "port",
            "sample": f"{n_crops} crops ({iters} ICP updates), scipy cKDTree + numpy SVD Umeyama (Open3D's loop shape)",
            "seconds": round(dt, 3)}


def main():
    cmd = launcher_cmd(sys.argv[1:], os.environ)
    if cmd is not None:  # --gpus N > 1 without a launcher: N ranks as a child job
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        sys.exit(subprocess.call(cmd, env=env))
    args = parse()
    if os.environ.get("PK_DEV") == "1":  # development runs only: libposekern_dev.so and its PK_* knobs
        from dpfm_amd import _lib as _devl
        _devl.use_dev_lib()
    world, rank, dev = setup_dist(args.gpus)
    apply_global_batch(args, world)
    from dpfm_amd import _lib
    build = {"train": build_train, "infer": build_infer, "corr4096": build_corr, "icp": build_icp,
             "ransac_ref": build_ransac_ref,
             "teaser": build_teaser, "operators": build_operators}[args.mode]
    one_step, probe_step, metric, units, config = build(args, dev, rank, world)

    for _ in range(args.warmup):
        one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    probe = KernelProbe()
    if args.eager:
        _lib.set_probe(probe.hook)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        log = one_step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    _lib.set_probe(None)
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if hasattr(one_step, "flush"):  # PipelinedTrainer: the last step's IR (computed beside the next step)
        one_step.flush()
        torch.cuda.synchronize()
    extra = {}
    # index consumers' per-crop status (IR / RANSAC met an out-of-range index; 0 expected), read
    # after timing like pair_overflow
    ist = log.get("ir_index_status" if args.mode == "train" else "index_status") if isinstance(log, dict) else None
    if ist is not None:
        extra["index_status_bad_crops"] = int((ist != 0).sum())
    if args.mode == "train":
        extra = {"loss": round(float(log["loss"]), 5), "ir": round(float(log["IR"]), 5),
                 "pair_overflow": bool(log["pair_overflow"])}
    elif args.mode == "infer":
        extra = {"mean_ir": round(float(log["ir"].mean()), 5), "mean_corr": round(float(log["n_corr"].float().mean()), 1)}
    elif args.mode == "operators":
        extra = {"operators": log}
    elif args.mode == "teaser":
        info = log["info"]
        extra = {"teaser": {"valid": int(info[:, 0].sum()), "kcore_heuristic": int((info[:, 1] == 2).sum()),
                            "exact": int((info[:, 1] == 1).sum()), "mean_clique": round(float(log["size"].mean()), 1),
                            "mean_rotation_inliers": round(float(info[:, 2].mean()), 1)}}
    elif args.mode == "icp":
        st = log["stats"].cpu().numpy()
        extra = {"icp": {"mean_fitness": round(float(st[:, 0].mean()), 5), "mean_rmse": round(float(st[:, 1].mean()), 6),
                         "mean_updates": round(float(st[:, 2].mean()), 2), "max_updates": int(st[:, 2].max()),
                         "converged": int(st[:, 3].sum())}}
    probe_steps = args.steps
    if not args.eager:
        # per-kernel HIP events cannot sit inside a graph: time the same step eagerly, on
        # the same resident inputs, right after the timed region (not part of `value`)
        # A device-side sleep heads each probe step so the host enqueues the whole step
        # before the GPU starts it: the events then bracket device time only, not host
        # launch gaps (an eager step is host-bound).
        _lib.set_probe(probe.hook)
        for _ in range(args.probe_steps):
            torch.cuda.synchronize()
            torch.cuda._sleep(int(2.5e8))  # ~0.1 s of GPU clock cycles
            probe_step()
        torch.cuda.synchronize()
        _lib.set_probe(None)
        probe_steps = args.probe_steps
    kern = probe.summary()

    if rank == 0:
        total_ms = elapsed * 1e3 / args.steps
        # dominant kernel family on the critical path: in the pipelined training execution crop
        # formation runs on a second stream under the training step, so the training kernels
        # bound the step; the crop-formation families are reported beside it
        overlapped = args.mode in ("train", "infer") and not args.no_overlap and not args.eager
        main_k = {k: v for k, v in kern.items() if not (overlapped and k in CROP_FAMS)} or kern
        # device families only: an entry point without declared work is host code (the f1 flip
        # stage pk_tufted_laplacian, the f2 clique / GNC solve), reported in `kernels`, not as a roofline
        main_k = {k: v for k, v in main_k.items() if v["work"] is not None} or main_k
        dom = max(main_k.items(), key=lambda kv: kv[1]["total_ms"]) if main_k else None
        crop_k = {k: v for k, v in kern.items() if k in CROP_FAMS}
        dom_crop = max(crop_k.items(), key=lambda kv: kv[1]["total_ms"]) if crop_k else None
        kernels = {k: {"avg_ms": round(v["avg_ms"], 4), "launches": v["launches"],
                       "ms_per_step": round(v["total_ms"] / max(probe_steps, 1), 4)}
                   for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"])}
        roof = roofline_for(dom[0], dom[1]) if dom is not None else None  # None: --probe-steps 0
        mfma_fams = {k: roofline_for(k, v) for k, v in kern.items() if v["bound"] in ("mfma", "mfma_bf16")}
        out = {
            "metric": metric,
            "value": round(units * world / elapsed * args.steps, 3),
            "unit": {"corr4096": "solves/s", "icp": "refinements/s", "teaser": "solves/s",
                     "operators": "operator sets/s", "ransac_ref": "solves/s"}.get(args.mode, "crops/s"),
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(total_ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if (args.mode == "corr4096" and args.fd_precision != "fp32") else "fp32",
            "data": "synthetic (seeded ellipsoid RGB-D frames, random-init DPFM)",
            "config": config,
            "roofline": roof,
            "roofline_crop_formation": (dict(roofline_for(dom_crop[0], dom_crop[1]),
                                             stream="side (overlapped with the main step)")
                                        if dom_crop is not None and overlapped else
                                        (roofline_for(dom_crop[0], dom_crop[1]) if dom_crop else None)),
            "roofline_mfma_kernels": {k: {"achieved": v["achieved"], "frac": v["frac"], "unit": v["unit"]}
                                      for k, v in mfma_fams.items()},
            "kernels": kernels,
        }
        out.update(extra)
        if "pk_ransac" in kern and args.mode in ("infer", "corr4096", "ransac_ref"):
            rk = kern["pk_ransac"]
            crops_per_launch = 1 if args.mode == "corr4096" else units
            if args.mode == "ransac_ref":
                args.hypotheses = config["hypotheses"]
            r64 = roofline_for("pk_ransac", rk)
            out["ransac"] = {"hypotheses_per_s": round(args.hypotheses * crops_per_launch / (rk["avg_ms"] * 1e-3), 1),
                             "ms_per_launch": round(rk["avg_ms"], 4), "hypotheses_per_launch":
                             args.hypotheses * crops_per_launch, "valu64_achieved_tflops": r64["achieved"],
                             "valu64_frac": r64["frac"]}
        if args.mode == "train" and not args.no_roofline_probe and world == 1:
            out["roofline_ball_query"] = ball_query_roofline(dev)
            out["roofline_feat_dist"] = feat_dist_roofline(dev)
        if args.mode == "infer" and not args.no_roofline_probe and world == 1 and args.points == 1024:
            # the configured solver's top-5 timed as the pipeline issues it (graph replays, warm
            # clocks); roofline_mfma_kernels' entry is the eager per-op probe (host gaps included)
            out["roofline_feat_dist_top5"] = feat_dist_roofline(dev, topk=5)
        if not args.no_cpu_baseline and world == 1 and not args.ragged:
            if args.mode == "train":
                out["cpu_baseline"] = cpu_baseline(args.cpu_crops, args.points, args.points)
                if args.pose_crops > 0:
                    out["pose_err"] = pose_real_check(dev, H=args.hypotheses)
                    if "fn" in POSE_CHECK:  # the model path on the synthetic batch (random-init weights)
                        out["pose_err"]["model_path"] = POSE_CHECK["fn"](args.pose_crops)
            elif args.mode == "corr4096":
                out["cpu_baseline"] = cpu_ransac_baseline(args.hypotheses)
            elif args.mode == "ransac_ref":
                out["cpu_baseline"] = cpu_ransac_baseline(config["hypotheses"], V=args.cad_points, n=760,
                                                          sample_h=200_000)
            elif args.mode == "icp":
                out["cpu_baseline"] = cpu_icp_baseline(32, args.icp_target)
            elif args.mode == "teaser":
                out["cpu_baseline"] = cpu_teaser_baseline(8, args.teaser_n)
            elif args.mode == "operators":
                out["cpu_baseline"] = cpu_ops_baseline(2, args.op_points)
            elif args.mode == "infer":
                out["cpu_baseline"] = cpu_infer_baseline(max(1, args.cpu_crops // 3), args.points, args.points,
                                                         args.hypotheses)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_ransac_baseline(H: int, V: int = 4096, sample_h: int = 0, n: int = 0) -> dict:
    """configs[4]'s pose stage on the host: the C/OpenMP restatement of Open3D 0.17's
    RegistrationRANSACBasedOnCorrespondence loop (oracle/c/oracle.c oc_ransac_o3d: per
    hypothesis a 4-point Umeyama, the WHOLE source cloud transformed as Open3D's loop does, the
    correspondences scored), on the same 4096-vertex CAD / 4096 correspondences; H hypotheses
    timed, the reference's 4x10^6 extrapolated linearly (stated as such)."""
    import ctypes
    from dpfm_amd.dataset.synthetic import random_rotation
    so = os.path.join(ROOT, "oracle", "build", "liboracle.so")
    lib = ctypes.CDLL(so)
    P = ctypes.c_void_p
    lib.oc_ransac_o3d.argtypes = [P, ctypes.c_int, P, P, ctypes.c_int, P, ctypes.c_uint64, ctypes.c_int64,
                                  ctypes.c_double, P, P]
    threads = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    os.environ["OMP_NUM_THREADS"] = str(threads)
    rng = np.random.default_rng(4096)
    cad = np.ascontiguousarray(rng.normal(size=(V, 3)) * 6)
    R = random_rotation(rng)
    pc = np.ascontiguousarray((cad[rng.permutation(V)] + rng.normal(size=(V, 3)) * 0.02) @ R.T + np.array([2.0, -1.0, 90.0]))
    n = n or V
    corres = np.ascontiguousarray(np.stack([rng.integers(0, V, n), np.arange(n)], 1).astype(np.int32))
    T, st = np.zeros(16), np.zeros(3)
    cp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    h = sample_h or H
    lib.oc_ransac_o3d(cp(cad), V, cp(pc), cp(corres), n, None, 0, 64, 0.05, cp(T), cp(st))  # warm-up
    t0 = time.perf_counter()
    lib.oc_ransac_o3d(cp(cad), V, cp(pc), cp(corres), n, None, 0, h, 0.05, cp(T), cp(st))
    dt = time.perf_counter() - t0
    import platform
    return {"value": round(1.0 / (dt * H / h), 4), "unit": "solves/s (RANSAC stage only, H = %d)" % H,
            "cores": threads, "kind": "port",
            "sample": f"{h} hypotheses x {n} correspondences, {V}-vertex source transformed per hypothesis "
                      f"(Open3D's loop), C/OpenMP on {platform.processor() or 'host'}",
            "seconds": round(dt, 3),
            "reference_4e6_hypotheses_s_extrapolated": round(dt * 4e6 / h, 1)}


def pmc_traffic(name: str):
    """HBM bytes per launch of a kernel family from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, made by tools/pmc_summary.py from separate FETCH_SIZE and
    WRITE_SIZE runs of this benchmark), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            v = json.load(f).get(name)
    except (OSError, ValueError):
        return None
    return None if v is None else round(v["traffic_bytes_per_launch"], 1)


def roofline_for(name: str, k: dict) -> dict:
    """Roofline of one kernel family from the probe: achieved = its declared algorithmic
    work (bytes for HBM-bound kernels, flops for MFMA kernels) summed over
    its launches / its summed launch time."""
    base = {"kernel": name, "avg_ms": round(k["avg_ms"], 4), "launches_per_step_probe": k["launches"],
            "work_per_launch": None if k["work"] is None else k["work"] / k["launches"]}
    traffic = pmc_traffic(name)
    layer_pmc = None
    if name in ("pk_linear_fwd", "pk_linear_ex"):
        # the counters cannot split the two entry points (same kernels): report the combined
        # per-kernel-launch bytes beside the roofline instead of as this family's traffic
        v = pmc_traffic("pk_linear_fwd+ex")
        layer_pmc = None if v is None else {"family": "pk_linear_fwd+ex", "bytes_per_kernel_launch": v,
                                             "note": "PMC FETCH+WRITE per per-point-layer kernel launch of both "
                                                     "entry points (profiles/pmc_traffic.json)"}
    if k["work"] is None:
        return dict(base, bound="hbm", achieved=None, peak=HBM_PEAK_GBS, unit="GB/s", frac=None, traffic=traffic)
    sec = k["total_ms"] * 1e-3
    if k["bound"] in ("mfma", "mfma_bf16"):
        ach = k["work"] / sec / 1e12
        peak = F32_MFMA_TFLOPS if k["bound"] == "mfma" else BF16_MFMA_TFLOPS
        r = dict(base, bound="mfma", achieved=round(ach, 3), peak=peak, unit="TFLOP/s",
                 frac=round(ach / peak, 4), traffic=traffic)
        if k["bound"] == "mfma_bf16":
            r["dtype"] = "bf16"
    elif k["bound"] in ("valu32", "valu64"):
        ach = k["work"] / sec / 1e12
        peak = F32_VALU_TFLOPS if k["bound"] == "valu32" else F64_VALU_TFLOPS
        r = dict(base, bound=k["bound"], achieved=round(ach, 3), peak=peak, unit="TFLOP/s",
                 frac=round(ach / peak, 4), traffic=traffic)
    else:
        ach = k["work"] / sec / 1e9
        r = dict(base, bound="hbm", achieved=round(ach, 2), peak=HBM_PEAK_GBS, unit="GB/s",
                 frac=round(ach / HBM_PEAK_GBS, 6), traffic=traffic)
    if k.get("flops") is not None:  # HBM-bound family that also declares its MFMA flops
        r["mfma_achieved_tflops"] = round(k["flops"] / sec / 1e12, 3)
        r["mfma_frac"] = round(k["flops"] / sec / 1e12 / F32_MFMA_TFLOPS, 4)
        r["note"] = ("per-point layers: 2 Cin Cout flop per 4 (Cin + Cout) B of a point, <= 21 flop/B, at or "
                     "below the f32 MFMA ridge (157.3 / 8 = 19.7 flop/B): bound by HBM; "
                     "each launch moves 4-50 MB, so launch ramp and tail are a large share")
    if name == "pk_fps":
        r["note"] = ("sequential npoint-step argmax, one workgroup per crop: latency-bound; the HBM "
                     "fraction is reported for completeness, not as its limiter")
    if layer_pmc is not None:
        r["pmc_layer_kernels"] = layer_pmc
    return r


if __name__ == "__main__":
    main()
