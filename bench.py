"""Headline benchmark: RGB-D crops/sec (fwd+bwd), 1024-point crops, per BASELINE.json.

One step = one training iteration of the reference (scripts/train.py:88-124) for a batch
of B synthetic 640x480 RGB-D frames, with the dataset's crop formation on the device:
  back-projection + erosion -> SOR kNN-20 -> FPS to 1024 -> align transform -> ball
  query (P, overlaps) -> RGB at the crop points -> DPFMNet fwd -> C_gt + DPFMLoss ->
  naive point map + inlier ratio -> backward -> grad all-reduce (N > 1) -> clip -> RMSprop.
Inputs (frames, CAD models, cached spectral operators) are resident in HBM before timing.

  python bench.py [--gpus N --steps K --warmup W --batch B]
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32, help="crops per GPU (configs[1]: 32)")
    ap.add_argument("--points", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-crops", type=int, default=30, help="bounded CPU-baseline sample (crops)")
    ap.add_argument("--no-roofline-probe", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no HIP graph: launch every kernel from Python")
    ap.add_argument("--no-overlap", action="store_true",
                    help="graph mode without overlapping crop formation of the next batch")
    ap.add_argument("--probe-steps", type=int, default=2, help="eager steps after timing for the kernel breakdown")
    return ap.parse_args()


class KernelProbe:
    """HIP events around every libposekern call (same stream as the kernels: torch's
    current stream), with the algorithmic work each launch declares (ops.py `work=`)."""

    def __init__(self):
        self.ev = {}

    def hook(self, name, fn, work=None):
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
            works = [w for _, _, w in lst]
            known = all(w is not None for w in works)
            out[k] = dict(avg_ms=float(np.mean(ms)), launches=len(ms), total_ms=float(np.sum(ms)),
                          bound=works[0][0] if known else None,
                          work=float(sum(w[1] for w in works)) if known else None,
                          flops=float(sum(w[2] for w in works)) if known and all(len(w) > 2 for w in works) else None)
        return out


def ball_query_roofline(dev, probe_launches: int = 10) -> dict:
    """pk_ball_query_mask at configs[3] size (B=256 crops, 2048 x 2048): >= 1 GB per launch."""
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
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(probe_launches):
        f()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / probe_launches
    byts = B * (24 * N + 24 * N + N * N) + B * N * 4  # coords in + mask + row counts
    ach = byts / (ms * 1e-3) / 1e9
    return {"kernel": "pk_ball_query_mask (configs[3]: 256 x 2048 x 2048)", "bound": "hbm", "achieved": round(ach, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
            "traffic": pmc_traffic("pk_ball_query_mask@configs3_probe"),
            "ms_per_launch": round(ms, 4), "bytes_per_launch": byts}


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
    t0 = time.perf_counter()
    for c in range(-1, n_crops):  # crop -1: untimed warm-up (allocator, thread pool)
        if c == 0:
            t0 = time.perf_counter()
        cs = c % 10_000  # non-negative seeds for the warm-up crop
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
    dt = time.perf_counter() - t0
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
    return {"value": round(n_crops / dt, 4), "unit": "crops/s (fwd+bwd incl. crop formation)", "cores": threads,
            "kind": "port",
            "sample": f"{n_crops} crops after 1 warm-up, {n2} pts, CAD {n1}; oracle/ (numpy + torch-CPU fp32) on {model_name}",
            "seconds": round(dt, 2)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
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

    from dpfm_amd import _lib
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedTrainStep, PipelinedTrainer, TrainStep, make_frame_batch

    B, N = args.batch, args.points
    torch.manual_seed(1234)  # identical initial weights on every rank (DDP broadcast semantics)
    model = DPFMNet().to(dev)
    fb, op = make_frame_batch(B, N, N, seed=1000 * rank, device=dev)
    crops_of = CropFormation(n1=N, npoint=N, seed=rank)
    step = TrainStep(model, seed=rank, capturable=not args.eager)

    if args.eager:
        def one_step():
            return step(op, crops_of(fb))
    elif args.no_overlap:  # warm-up + capture (untimed), then every step is a graph replay
        one_step = GraphedTrainStep(crops_of, step, fb, op, warmup=3)
    else:  # same, with crop formation of the next batch on a second stream
        one_step = PipelinedTrainer(crops_of, step, fb, op, warmup=3)

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
    loss_v, ir_v = float(log["loss"]), float(log["IR"])
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
            step(op, crops_of(fb))
        torch.cuda.synchronize()
        _lib.set_probe(None)
        probe_steps = args.probe_steps
    kern = probe.summary()

    if rank == 0:
        total_ms = elapsed * 1e3 / args.steps
        # dominant kernel family on the critical path: in the pipelined execution crop
        # formation runs on a second stream under the training step, so the training
        # kernels bound the step; the crop-formation families are reported beside it
        crop_fams = {"pk_backproject", "pk_sor", "pk_fps_npoint", "pk_fps", "pk_gather_transform",
                     "pk_ball_query_mask", "pk_ball_query_pairs", "pk_sample_rgb", "pk_erode_mask"}
        train_k = {k: v for k, v in kern.items() if k not in crop_fams} or kern
        dom = max(train_k.items(), key=lambda kv: kv[1]["total_ms"]) if train_k else None
        crop_k = {k: v for k, v in kern.items() if k in crop_fams}
        dom_crop = max(crop_k.items(), key=lambda kv: kv[1]["total_ms"]) if crop_k else None
        kernels = {k: {"avg_ms": round(v["avg_ms"], 4), "launches": v["launches"],
                       "ms_per_step": round(v["total_ms"] / max(probe_steps, 1), 4)}
                   for k, v in sorted(kern.items(), key=lambda kv: -kv[1]["total_ms"])}
        roof = roofline_for(dom[0], dom[1]) if dom is not None else None  # None: --probe-steps 0
        mfma_fams = {k: roofline_for(k, v) for k, v in kern.items() if v["bound"] == "mfma"}
        out = {
            "metric": "RGB-D crops/sec (fwd+bwd), 1024 pts, at 1/2/4/8 MI355X; pose err vs ref",
            "value": round(B * world / elapsed * args.steps, 3),
            "unit": "crops/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(total_ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp32", "data": "synthetic (seeded ellipsoid RGB-D frames, random-init DPFM)",
            "config": {"workload": "configs[1] shape: B=32 synthetic 640x480 RGB-D crops/GPU, 1024 pts, "
                                   "training step fwd+bwd (configs[2] semantics, DDP over RCCL when N>1)",
                       "execution": "eager" if args.eager else ("hip-graph" if args.no_overlap else
                                                                 "hip-graph, crop formation overlapped"),
                       "global_batch": B * world, "points_per_crop": N, "cad_points": N,
                       "precision": "model fp32 (f32 MFMA); crop geometry / C_gt normal equations fp64",
                       "parallelism": f"dp{world}"},
            "roofline": roof,
            "roofline_crop_formation": (dict(roofline_for(dom_crop[0], dom_crop[1]),
                                             stream="side (overlapped with the training step)")
                                        if dom_crop is not None and not args.no_overlap and not args.eager else
                                        (roofline_for(dom_crop[0], dom_crop[1]) if dom_crop else None)),
            "roofline_mfma_kernels": {k: {"achieved": v["achieved"], "frac": v["frac"], "unit": v["unit"]}
                                      for k, v in mfma_fams.items()},
            "kernels": kernels,
            "loss": round(loss_v, 5), "ir": round(ir_v, 5),
        }
        if not args.no_roofline_probe and world == 1:
            out["roofline_ball_query"] = ball_query_roofline(dev)
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_crops, N, N)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


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
    if k["work"] is None:
        return dict(base, bound="hbm", achieved=None, peak=HBM_PEAK_GBS, unit="GB/s", frac=None, traffic=traffic)
    sec = k["total_ms"] * 1e-3
    if k["bound"] == "mfma":
        ach = k["work"] / sec / 1e12
        r = dict(base, bound="mfma", achieved=round(ach, 3), peak=F32_MFMA_TFLOPS, unit="TFLOP/s",
                 frac=round(ach / F32_MFMA_TFLOPS, 4), traffic=traffic)
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
    return r


if __name__ == "__main__":
    main()
