"""The hot path end to end on the device: RGB-D frames -> crops -> DPFM fwd(+bwd) ->
correspondences -> pose.

  make_frame_batch   seeded synthetic frames / CAD / spectral operators resident in HBM
  TrainStep          one iteration of scripts/train.py:88-124 for a batch of crops:
                     model fwd, C_gt (utils/utils.py:67-79), DPFMLoss, the per-crop naive
                     point map + inlier ratio (train.py:109-116), backward, gradient
                     all-reduce across ranks (DDP semantics, one bucket), clip 5.0, RMSprop
  InferStep          scripts/eval.py:57-119 + scripts/test_RANSAC.py:397-419 for a batch:
                     model fwd, spatial-filtering solver, IR, RANSAC pose, pose metrics
Nothing here synchronises with the host; callers decide when to read results.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib, ops
from .dataset.object import CropFormation, Crops, FrameBatch
from .dataset.synthetic import cad_points, lbo_operators, make_frame
from .models.dpfm import DPFMNet
from .layers import Conv1d, GroupedWgrad, Linear
from .diffusion_net import LearnedTimeDiffusion
from .utils.loss import DPFMLoss


@dataclass
class Operators:
    """Cached spectral operators (the reference's CAD_LBO / pc_LBO npz caches)."""
    cad_mass: torch.Tensor   # f32 [F, N1]
    cad_evals: torch.Tensor  # f32 [F, 64]
    cad_evecs: torch.Tensor  # f32 [F, N1, 64]
    cad_xyz: torch.Tensor    # f32 [F, N1, 3]
    pc_mass: torch.Tensor    # f32 [F, N2]
    pc_evals: torch.Tensor   # f32 [F, 64]
    pc_evecs: torch.Tensor   # f32 [F, N2, 64]
    ir_thr: torch.Tensor     # f32 [F] 0.1 * diam (train.py:115)
    rig_thr: torch.Tensor    # f32 [F, 4] spatial-filter thresholds
    cad_n: Optional[torch.Tensor] = None  # int32 [F] CAD vertices per crop (rows of cad_* not padding)
    pc_spectral: Optional[object] = None  # geometry.SpectralOperators the pc_* fields came from (f1 path)


def pad_rows(arrs, ld: Optional[int] = None) -> np.ndarray:
    """collate's pad_sequence on host arrays: stack along a new batch axis, zero-padding the
    first axis to `ld` (default: the longest)."""
    ld = max(a.shape[0] for a in arrs) if ld is None else ld
    out = np.zeros((len(arrs), ld) + arrs[0].shape[1:], dtype=arrs[0].dtype)
    for b, a in enumerate(arrs):
        out[b, :a.shape[0]] = a
    return out


def crop_operators(op: Operators, crops: Crops, seed: int) -> Operators:
    """Operators whose crop part matches the formed crops' true sizes: per crop the cached
    pc_LBO of a crop of n2 points (dataset/object.py:240-269; the synthetic stand-in of
    lbo_operators), zero-padded to crops.ld as collate pads them. Reads the crop sizes
    (host sync): the reference computes these operators per crop, offline, from the crop."""
    counts = crops.n2.cpu().numpy().tolist()
    dev = crops.pc32.device
    ops_p = [lbo_padded(int(n), 2 * (seed + b) + 1) for b, n in enumerate(counts)]
    pm = torch.as_tensor(pad_rows([o[0] for o in ops_p], crops.ld), device=dev)
    pv = torch.as_tensor(pad_rows([o[2] for o in ops_p], crops.ld), device=dev)
    pe = torch.as_tensor(np.stack([o[1] for o in ops_p]), device=dev)
    return Operators(cad_mass=op.cad_mass, cad_evals=op.cad_evals, cad_evecs=op.cad_evecs, cad_xyz=op.cad_xyz,
                     pc_mass=pm, pc_evals=pe, pc_evecs=pv, ir_thr=op.ir_thr, rig_thr=op.rig_thr, cad_n=op.cad_n)


def device_crop_operators(op: Operators, crops: Crops, k_eig: int = 64, **eig_kw) -> Operators:
    """The (f1) new-crop path: the crops' spectral operators computed on the device from the formed
    crop points themselves (dataset/object.py:246 get_operators(verts=torch.Tensor(pcd_depth),
    faces=[], k_eig=64): the reference rounds the crop to f32 first, so does this), zero-padded to
    crops.ld as collate pads them; the CAD part of `op` is kept (the reference caches it per
    object). Chains crop formation -> operators -> DPFMNet -> pose without the offline cache.
    Reads the crop sizes (host sync: the eigensolver's subspace width depends on them)."""
    from . import geometry
    counts = crops.n2.cpu().tolist()
    pts = crops.pc64.float().double()
    so = geometry.point_cloud_operators(pts, crops.off, counts, k_eig=k_eig, **eig_kw)
    F, ld, nm = len(counts), crops.ld, so.evecs.shape[1]
    dev = crops.pc32.device
    pv = torch.zeros(F, ld, k_eig, dtype=torch.float32, device=dev)
    pv[:, :nm] = so.evecs.float()
    pm = torch.zeros(F, ld, dtype=torch.float32, device=dev)
    pm[:, :nm] = so.mass.float()
    return Operators(cad_mass=op.cad_mass, cad_evals=op.cad_evals, cad_evecs=op.cad_evecs, cad_xyz=op.cad_xyz,
                     pc_mass=pm, pc_evals=so.evals.float().contiguous(), pc_evecs=pv, ir_thr=op.ir_thr,
                     rig_thr=op.rig_thr, cad_n=op.cad_n, pc_spectral=so)


def make_frame_batch(F: int, n1: int, n2: int, seed: int, device) -> tuple[FrameBatch, Operators]:
    depth, mask, rgb, K, cs, R, t, cad, diam = [], [], [], [], [], [], [], [], []
    ops_c, ops_p = [], []
    maxpix = 0
    for f in range(F):
        fr = make_frame(seed + f)
        depth.append(fr.depth.view(np.int16))
        mask.append(fr.mask)
        rgb.append(fr.rgb)
        K.append(fr.K.reshape(9))
        cs.append(np.float32(1000.0 / fr.depth_scale))
        R.append(fr.R_m2c.reshape(9))
        t.append(fr.t_m2c)
        cad.append(cad_points(fr, n1, seed + f))
        diam.append(fr.diam_cad)
        maxpix = max(maxpix, int((fr.mask == 255).sum()))
        ops_c.append(lbo_operators(n1, 64, 2 * (seed + f)))
        ops_p.append(lbo_operators(n2, 64, 2 * (seed + f) + 1))
    d = torch.device(device)
    T = lambda a, dt=None: torch.as_tensor(np.stack(a), device=d) if dt is None else torch.as_tensor(np.stack(a), dtype=dt, device=d)  # noqa: E731
    fb = FrameBatch(depth=T(depth), mask=T(mask), rgb=T(rgb), K=T(K, torch.float64), cam_scale=T(cs, torch.float32),
                    R=T(R, torch.float64), t=T(t, torch.float64),
                    cad64=torch.as_tensor(np.concatenate(cad, 0), dtype=torch.float64, device=d),
                    cad_off=ops.packed_offsets([n1] * F, d), diam=diam, max_pixels=maxpix,
                    thr2=torch.tensor([ops.ball_threshold(0.05 * x) for x in diam], dtype=torch.float64, device=d),
                    n1max=n1)
    # CAD and crop operators of the batch in ONE buffer each ([CAD; crops] along the batch):
    # the model's shared encoder pass over both shapes then needs no concatenation copy
    def joint(k):
        if ops_c[0][k].shape != ops_p[0][k].shape:  # n1 != n2: separate buffers
            return T([o[k] for o in ops_c]), T([o[k] for o in ops_p])
        both = T([o[k] for o in ops_c] + [o[k] for o in ops_p])
        return both[:F], both[F:]
    (cm, pm), (ce, pe), (cv, pv) = joint(0), joint(1), joint(2)
    op = Operators(cad_mass=cm, cad_evals=ce, cad_evecs=cv, cad_xyz=T([c.astype(np.float32) for c in cad]),
                   pc_mass=pm, pc_evals=pe, pc_evecs=pv,
                   ir_thr=torch.tensor([np.float32(0.1 * x) for x in diam], dtype=torch.float32, device=d),
                   rig_thr=ops.rigidity_thresholds(diam, d),
                   cad_n=torch.full((F,), n1, dtype=torch.int32, device=d))
    return fb, op


def frame_batch(frames: list, device) -> FrameBatch:
    """FrameBatch from per-frame dicts with the fields the reference's datasets read
    (dataset/scene.py:125-158, object.py:133-164): depth uint16 [H, W], mask uint8 [H, W]
    (mask_visib, 255 = object), K [3, 3], depth_scale, R_m2c [3, 3], t_m2c [3] (cm), cad f64
    [n1, 3] (cm, the decimated CAD vertices; ragged across frames), diam_cad (cm); rgb uint8
    [H, W, 3] optional."""
    d = torch.device(device)
    st = lambda key, dt: torch.as_tensor(np.stack([np.asarray(f[key], dtype=dt) for f in frames]), device=d)  # noqa
    H, W = np.asarray(frames[0]["depth"]).shape[:2]
    rgb = [np.asarray(f["rgb"], dtype=np.uint8) if f.get("rgb") is not None else np.zeros((H, W, 3), np.uint8)
           for f in frames]
    cads = [np.asarray(f["cad"], dtype=np.float64).reshape(-1, 3) for f in frames]
    diam = [float(f["diam_cad"]) for f in frames]
    return FrameBatch(
        depth=torch.as_tensor(np.stack([np.asarray(f["depth"], dtype=np.uint16).view(np.int16) for f in frames]),
                              device=d),
        mask=st("mask", np.uint8), rgb=torch.as_tensor(np.stack(rgb), device=d),
        K=torch.as_tensor(np.stack([np.asarray(f["K"], np.float64).reshape(9) for f in frames]), device=d),
        cam_scale=torch.tensor([np.float32(1000.0 / f["depth_scale"]) for f in frames], dtype=torch.float32,
                               device=d),
        R=torch.as_tensor(np.stack([np.asarray(f["R_m2c"], np.float64).reshape(9) for f in frames]), device=d),
        t=torch.as_tensor(np.stack([np.asarray(f["t_m2c"], np.float64).reshape(3) for f in frames]), device=d),
        cad64=torch.as_tensor(np.concatenate(cads, 0), device=d), cad_off=ops.packed_offsets([len(c) for c in cads], d),
        diam=diam, max_pixels=max(int((np.asarray(f["mask"]) == 255).sum()) for f in frames),
        thr2=torch.tensor([ops.ball_threshold(0.05 * x) for x in diam], dtype=torch.float64, device=d),
        n1max=max(len(c) for c in cads))


def lbo_padded(n: int, seed: int, k: int = 64):
    """Synthetic stand-in of one shape's cached LBO operators (mass [n], evals [k], evecs
    [n, k]); fewer than k points leave the missing eigenvectors as zero columns."""
    m, e, v = lbo_operators(max(n, 1), k, seed)
    if v.shape[1] < k:
        v = np.concatenate([v, np.zeros((v.shape[0], k - v.shape[1]), np.float32)], 1)
    return m[:n], e, v[:n]


def operators_for(cads: list, crop_counts: list, diam: list, seed: int, device, ld2: Optional[int] = None) -> Operators:
    """Operators of a ragged batch, padded as collate pads them: CAD b (f64 [n1_b, 3], cm)
    with lbo_padded(n1_b, 2 (seed + b)), crop b with lbo_padded(n2_b, 2 (seed + b) + 1)."""
    d = torch.device(device)
    oc = [lbo_padded(len(c), 2 * (seed + b)) for b, c in enumerate(cads)]
    op_ = [lbo_padded(int(n), 2 * (seed + b) + 1) for b, n in enumerate(crop_counts)]
    T = lambda a: torch.as_tensor(a, device=d)  # noqa: E731
    return Operators(cad_mass=T(pad_rows([o[0] for o in oc])), cad_evals=T(np.stack([o[1] for o in oc])),
                     cad_evecs=T(pad_rows([o[2] for o in oc])),
                     cad_xyz=T(pad_rows([np.asarray(c, np.float64).astype(np.float32) for c in cads])),
                     pc_mass=T(pad_rows([o[0] for o in op_], ld2)), pc_evals=T(np.stack([o[1] for o in op_])),
                     pc_evecs=T(pad_rows([o[2] for o in op_], ld2)),
                     ir_thr=torch.tensor([np.float32(0.1 * x) for x in diam], dtype=torch.float32, device=d),
                     rig_thr=ops.rigidity_thresholds(diam, d),
                     cad_n=torch.tensor([len(c) for c in cads], dtype=torch.int32, device=d))


def model_batch(op: Operators, crops: Crops) -> dict:
    """The {"shape1": CAD, "shape2": PC} dict of train.py:88-91 (L/grad operators None)."""
    cad = {"xyz": op.cad_xyz, "mass": op.cad_mass, "evals": op.cad_evals, "evecs": op.cad_evecs,
           "L": None, "gradX": None, "gradY": None, "faces": None}
    pc = {"xyz": crops.pc32, "mass": op.pc_mass, "evals": op.pc_evals, "evecs": op.pc_evecs,
          "L": None, "gradX": None, "gradY": None}
    return {"shape1": cad, "shape2": pc}


def _counts(n: Optional[torch.Tensor], B: int, full: int, dev) -> torch.Tensor:
    return n.to(torch.int32) if n is not None else torch.full((B,), full, dtype=torch.int32, device=dev)


def naive_p2p_batched(C: torch.Tensor, evecs_x: torch.Tensor, evecs_y: torch.Tensor,
                      n1: Optional[torch.Tensor] = None, n2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """naive_fmap2pointmap for every crop: int64 [B, 2, V2] (row 0 CAD idx, row 1 arange).
    n1 / n2 (int32 [B]): the rows of the padded evecs that are real points — train.py:110-114
    keeps the rows whose xyz is non-zero, i.e. drops collate's padding; entries j >= n2[b]
    of crop b are unspecified."""
    B, V1, _ = evecs_x.shape
    V2 = evecs_y.shape[1]
    dev = C.device
    n1 = _counts(n1, B, V1, dev)
    n2 = _counts(n2, B, V2, dev)
    idx, _ = ops.feat_dist_topk(evecs_x, C, evecs_y, n1, n2, 1)
    ar = torch.arange(V2, device=dev, dtype=torch.int64)[None].expand(B, V2)
    return torch.stack([idx[..., 0], ar], 1)


class TrainStep:
    """One training iteration (scripts/train.py:88-124) for a batch of crops.

    Split in two phases so a HIP graph can hold everything but the collective:
    `forward_backward` (model, C_gt, loss, naive IR, backward) and `apply` (gradient
    all-reduce across ranks, clip 5.0, RMSprop, grads reset to None as the next
    backward re-creates them)."""

    def __init__(self, model: DPFMNet, lr: float = 5e-4, max_norm: float = 5.0, nce_num_pairs: int = 512,
                 group: Optional[dist.ProcessGroup] = None, seed: int = 0, capturable: bool = False,
                 grouped: bool = True, fused_opt: bool = True):
        self.model = model
        self.params = [p for p in model.parameters()]
        # config/dpfm_orig.gin:62-63; capturable keeps the step count on the device
        self.opt = torch.optim.RMSprop(self.params, lr=lr, capturable=capturable)
        self.crit = DPFMLoss(w_fmap=1, w_acc=1, w_nce=1, nce_t=0.07, nce_num_pairs=nce_num_pairs)  # gin:54-58
        self.max_norm = max_norm
        self.group = group
        self.world = dist.get_world_size(group) if (group is not None or dist.is_initialized()) else 1
        dev = self.params[0].device
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        self.flat = torch.zeros(sum(p.numel() for p in self.params), dtype=torch.float32, device=dev)
        # HIP devices: every .grad is a view of `flat` (zeroed at the start of each backward),
        # so DDP's all-reduce is one collective on `flat` with no gather / scatter copies
        self.flat_grads = dev.type == "cuda"
        self.gviews = []
        o = 0
        for p in self.params:
            self.gviews.append(self.flat[o:o + p.numel()].view_as(p))
            o += p.numel()
        # clip + RMSprop in one HIP launch on HIP devices (torch's optimizer keeps the state)
        self.fused_opt = fused_opt and dev.type == "cuda" and len(self.params) <= 96
        # grouped=True (HIP devices): the per-point layers' weight gradients are recorded during
        # backward and computed in one grouped launch pair at its end (layers.GroupedWgrad).
        # The step stays on one stream: forking C_gt / the IR onto an auxiliary stream inside
        # the captured graph replayed ~1 ms/step slower on MI355X.
        self.side = None
        if grouped and dev.type == "cuda":
            lin = [p for m in model.modules() if isinstance(m, (Linear, Conv1d)) for p in m.parameters(recurse=False)]
            # gradients the fused encoder's kernels write whole into .grad (GroupedWgrad.direct): the
            # diffusion times (autograd's accumulation on the non-fused encoder path)
            dts = [m.diffusion_time for m in model.modules() if isinstance(m, LearnedTimeDiffusion)]
            self.side = GroupedWgrad(lin, bufs={id(p): v for p, v in zip(self.params, self.gviews)}
                                     if self.flat_grads else None, direct_params=dts)

    def nce_counter(self) -> torch.Tensor:
        """The device step counter keying this step's NCE pair draws (utils/loss.py)."""
        from .utils.loss import _NCE_CTR
        dev = self.params[0].device
        key = (id(self.gen), str(dev))
        if key not in _NCE_CTR:
            _NCE_CTR[key] = torch.zeros(1, dtype=torch.int64, device=dev)
        return _NCE_CTR[key]

    @torch.no_grad()
    def load_state_from(self, other: "TrainStep") -> None:
        """Copy parameters, optimizer state and the NCE draw counter of `other` in place
        (tensor storages are kept, so a captured graph over `self` stays valid)."""
        for p, q in zip(self.params, other.params):
            p.copy_(q)
        for p, q in zip(self.params, other.params):
            sp, sq = self.opt.state.get(p, {}), other.opt.state.get(q, {})
            for k, v in sq.items():
                if k in sp and torch.is_tensor(sp[k]):
                    sp[k].copy_(v)
                else:
                    sp[k] = v.clone() if torch.is_tensor(v) else v
            self.opt.state[p] = sp
        self.nce_counter().copy_(other.nce_counter())

    def allreduce_grads(self, grads=None, force: bool = False):
        """DDP's gradient averaging in one bucket (49,281 f32 = 197 KB: latency-bound).
        `grads` defaults to the parameters' .grad tensors. With one rank nothing runs unless
        `force` (the collective path on an initialised group of size 1: tests/_rccl_worker.py)."""
        if self.world <= 1 and not force:
            return
        if self.flat_grads:  # the gradients ARE views of flat: one collective, one scale
            dist.all_reduce(self.flat, group=self.group)
            if self.world > 1:
                self.flat.div_(self.world)
            return
        grads = grads if grads is not None else [p.grad for p in self.params]
        o = 0
        for g in grads:
            n = g.numel()
            self.flat[o:o + n].copy_(g.reshape(-1))
            o += n
        dist.all_reduce(self.flat, group=self.group)
        if self.world > 1:
            self.flat.div_(self.world)
        o = 0
        for g in grads:
            n = g.numel()
            g.copy_(self.flat[o:o + n].view_as(g))
            o += n

    @staticmethod
    @torch.no_grad()
    def ground_truth(op: Operators, crops: Crops) -> torch.Tensor:
        """C_gt of the crops (utils/utils.py:67-79): reads only P and the two bases, so a
        producer may form it with the crops (Crops.C_gt) off the step's critical path."""
        return ops.cgt_lstsq(crops.pairs, crops.npairs, op.cad_evecs, op.pc_evecs, cnt=crops.pair_cols)

    @staticmethod
    @torch.no_grad()
    def inlier_ratio_of(op: Operators, crops: Crops, C_pred: torch.Tensor,
                        status: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """train.py:109-116: the naive point map of C_pred and its mean inlier ratio over the
        crops (naive_p2p_batched without materialising its arange row: the IR kernel reads the
        map as [B, V2] CAD indices of crop points 0..n2-1)."""
        B_, V2_ = op.pc_evecs.shape[0], op.pc_evecs.shape[1]
        n1 = _counts(op.cad_n, B_, op.cad_evecs.shape[1], C_pred.device)
        npred = _counts(crops.n2, B_, V2_, C_pred.device)
        p_map, _ = ops.feat_dist_topk(op.cad_evecs, C_pred.detach(), op.pc_evecs, n1, npred, 1)
        # status (int32 [B], optional): per crop 1 when a point-map index was out of range
        ir = ops.inlier_ratio(p_map[..., 0], npred, op.cad_xyz, crops.align32, op.ir_thr, layout=2, status=status)
        return ops.mean_f32(ir, out=out)

    def forward_backward(self, op: Operators, crops: Crops, ir: bool = True) -> dict:
        """ir=False leaves the naive point map + IR out of the step (PipelinedTrainer computes it
        beside the next steps from the C_pred this step leaves in `self.last_C_pred`)."""
        self.model.train()
        batch = model_batch(op, crops)
        C_gt = crops.C_gt
        if C_gt is None:
            C_gt = self.ground_truth(op, crops)
        C_pred, o12, o21, f1, f2, _, _ = self.model(batch)
        self.last_C_pred = C_pred.detach()
        loss, log = self.crit.forward_batched(C_pred, C_gt, crops.pairs, crops.npairs, f1, f2, o12, o21,
                                              crops.overlap_12, crops.overlap_21, generator=self.gen)
        with torch.no_grad():  # train.py:109-116 (naive solver + IR per crop)
            st = torch.empty((C_pred.shape[0],), dtype=torch.int32, device=C_pred.device) if ir else None
            ir = self.inlier_ratio_of(op, crops, C_pred, status=st) if ir else None
            if st is not None:
                log["ir_index_status"] = st  # device int32 [B] (ops.check_index_status)
            # P truncated at the pair capacity would train on partial labels: flag it (device
            # bool, formed with the crops on the crop-formation stream)
            log["pair_overflow"] = crops.overflow()
        if self.flat_grads:  # accumulate into the flat buffer's views (autograd adds in place)
            self.flat.zero_()
            for p, v in zip(self.params, self.gviews):
                p.grad = v
        if self.side is not None:
            self.side.begin()
        ok = False
        if getattr(self, "_seed_grad", None) is None or self._seed_grad.device != loss.device:
            self._seed_grad = torch.ones((), dtype=loss.dtype, device=loss.device)  # persistent: no fill per step
        try:
            torch.autograd.backward(loss, grad_tensors=self._seed_grad)
            ok = True
        finally:
            if self.side is not None:
                self.side.end(run=ok)
        if ir is not None:
            log["IR"] = ir
        return log

    def _fused_state(self):
        """The optimizer's per-parameter state (RMSprop's lazy init: step, square_avg),
        created in place if missing, so torch's optimizer object keeps owning it."""
        steps, sqs = [], []
        for p in self.params:
            st = self.opt.state[p]
            if len(st) == 0:
                st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)
                st["square_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            steps.append(st["step"])
            sqs.append(st["square_avg"])
        return steps, sqs

    def apply(self, allreduce: bool = True, reset: bool = True):
        if allreduce:
            self.allreduce_grads()
        grp = self.opt.param_groups[0]
        fused = (self.fused_opt and len(self.opt.param_groups) == 1 and grp["momentum"] == 0 and not grp["centered"]
                 and grp["weight_decay"] == 0 and all(p.grad is not None for p in self.params))
        if fused:  # clip_grad_norm_ + RMSprop.step in one launch (pk_clip_rmsprop)
            steps, sqs = self._fused_state()
            ops.clip_rmsprop(self.params, [p.grad for p in self.params], sqs, steps, self.max_norm, grp["lr"],
                             grp["alpha"], grp["eps"])
        else:
            torch.nn.utils.clip_grad_norm_(self.params, max_norm=self.max_norm, norm_type=2)
            self.opt.step()
        if reset:  # (a captured backward that started from None grads overwrites them instead)
            self.opt.zero_grad(set_to_none=True)

    def __call__(self, op: Operators, crops: Crops):
        log = self.forward_backward(op, crops)
        self.apply()
        return log


class GraphedTrainStep:
    """Crop formation + a training step captured once into HIP graphs and replayed.

    The eager step issues ~700 launches (libposekern + torch); replaying a graph turns
    them into one submission, so the step runs at device speed. Inputs are static: `fb`
    and `op` stay resident and are re-read on every replay (copy new frames into them to
    feed new data). With one rank the whole step is one graph; with several ranks the
    RCCL all-reduce runs eagerly between graph A (crops -> backward) and graph B
    (clip + RMSprop), so no collective is captured."""

    def __init__(self, crop_formation: CropFormation, step: TrainStep, fb: FrameBatch, op: Operators,
                 warmup: int = 3):
        self.crops_of, self.step, self.fb, self.op = crop_formation, step, fb, op
        self.split = step.world > 1
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up outside capture (allocator, optimizer state)
            for _ in range(warmup):
                step.forward_backward(op, crop_formation(fb))
                step.apply()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph_a = torch.cuda.CUDAGraph()
        self.graph_a.register_generator_state(step.gen)
        # grads are None here, so the captured backward writes (not accumulates) them
        with torch.cuda.graph(self.graph_a):
            self.log = step.forward_backward(op, crop_formation(fb))
            if not self.split:
                step.apply(allreduce=False, reset=False)
        self.graph_b = None
        if self.split:
            self.graph_b = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph_b, pool=self.graph_a.pool()):
                step.apply(allreduce=False, reset=False)

    def __call__(self) -> dict:
        self.graph_a.replay()
        if self.split:
            self.step.allreduce_grads()
            self.graph_b.replay()
        return self.log


_MASKED_STREAMS = {}


def cu_split_streams(side_cus: int, device=None):
    """(main, side) torch streams over disjoint CU sets (pk_stream_create_cu_mask): `side_cus` CUs
    spread evenly over the device's CU index range for crop formation, the rest for the training
    (or inference) step, so the two never share a CU. Cached per (device, side_cus); the HIP
    streams live for the process."""
    import ctypes
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (str(dev), int(side_cus))
    if key in _MASKED_STREAMS:
        return _MASKED_STREAMS[key]
    n = ctypes.c_int(0)
    with torch.cuda.device(dev):
        _lib.call("pk_device_cu_count", ctypes.byref(n))
        ncu = int(n.value)
        if not 0 < side_cus < ncu:
            raise ValueError(f"side_cus must be in (0, {ncu})")
        words = (ncu + 31) // 32
        side_set = {min(ncu - 1, int((i + 0.5) * ncu / side_cus)) for i in range(side_cus)}
        masks = []
        for sel in (lambda c: c not in side_set, lambda c: c in side_set):
            m = (ctypes.c_uint32 * words)()
            for c in range(ncu):
                if sel(c):
                    m[c // 32] |= 1 << (c % 32)
            masks.append(m)
        out = []
        for m in masks:
            h = ctypes.c_void_p()
            _lib.call("pk_stream_create_cu_mask", m, words, ctypes.byref(h))
            out.append(torch.cuda.ExternalStream(h.value, device=dev))
    _MASKED_STREAMS[key] = tuple(out)
    return _MASKED_STREAMS[key]


class PipelinedTrainer:
    """Crop formation of batch i+1 overlapped with the training step on batch i.

    Crop formation (back-projection, SOR, FPS, ball query: ~2 ms of mostly latency-bound,
    one-workgroup-per-crop kernels at B = 32) and the model step (wide kernels) run on
    two streams, as the reference overlaps its DataLoader workers with training. Two
    crop buffers ping-pong: graph C_k forms crops into buffer k on the side stream, graph
    T_k trains on buffer k on the main stream; events order C_k after T_k of the previous
    use and T_k after C_k. Every piece is a HIP graph replay. With several ranks each
    T_k is split around the eager RCCL all-reduce, as in GraphedTrainStep.

    The step's naive point map + IR (a logged metric; nothing trains on it) leaves the training
    graphs (defer_ir=False keeps it there): graph I_k computes the IR of buffer k's batch from
    the C_pred that T_k left, on the crop-formation stream right before C_k overwrites the
    buffer. The log's "IR" tensor is filled in place by that side-stream graph, so a reader must
    be ordered after it: call wait_ir() (the current stream then waits for every IR enqueued so
    far: the logs of all calls but the last) or flush() (also computes the last call's IR)
    before reading log["IR"] on the device or the host.

    cgt_side=True solves C_gt with the crops on the crop-formation stream (the default since round
    5 keeps it in the training graph: with crop formation on the step's critical path that is
    0.9 % faster); side_cus > 0 puts the two streams on disjoint CU sets
    (cu_split_streams; measured no faster)."""

    def __init__(self, crop_formation: CropFormation, step: TrainStep, fb: FrameBatch, op: Operators,
                 warmup: int = 3, defer_ir: bool = True, cgt_side: bool = False, side_cus: int = 0,
                 main_priority: int = 0, side_after: bool = False):
        self.step, self.split = step, step.world > 1
        self.side_after = side_after  # host order per call: the training replay first, then crop formation
        self.main = torch.cuda.current_stream()
        self.side = torch.cuda.Stream()
        self.own_main = False
        if side_cus > 0:  # disjoint CU sets for the two streams (cu_split_streams)
            self.main, self.side = cu_split_streams(side_cus)
            self.main.wait_stream(torch.cuda.current_stream())
            self.own_main = True
        elif main_priority == 1:  # the training stream at the highest queue priority, crop formation below
            self.main = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
            self.main.wait_stream(torch.cuda.current_stream())
            self.own_main = True
        elif main_priority == -1:  # crop formation at the highest queue priority
            self.side = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
        side = torch.cuda.Stream()
        side.wait_stream(self.main)
        with torch.cuda.stream(side):  # warm-up outside capture
            for _ in range(warmup):
                step.forward_backward(op, crop_formation(fb))
                step.apply()
        self.main.wait_stream(side)
        torch.cuda.synchronize()
        self.crop_graphs, self.crops, self.train_a, self.train_b, self.grads, self.logs = [], [], [], [], [], []
        for k in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                c = crop_formation(fb)
                # C_gt depends only on the crops and the bases: solve it on the crop-formation
                # stream too (cgt_side=False keeps it in the training graph)
                if cgt_side:
                    c.C_gt = TrainStep.ground_truth(op, c)
                self.crops.append(c)
            self.crop_graphs.append(g)
        self.defer_ir = defer_ir
        self.ir_graphs, self._trained = [], [False, False]
        self.ir_done, self._ir_enqueued = [torch.cuda.Event(), torch.cuda.Event()], [False, False]
        for k in range(2):
            step.opt.zero_grad(set_to_none=True)  # each training graph owns its gradients
            ga = torch.cuda.CUDAGraph()
            ga.register_generator_state(step.gen)
            with torch.cuda.graph(ga):
                self.logs.append(step.forward_backward(op, self.crops[k], ir=not self.defer_ir))
                if not self.split:
                    step.apply(allreduce=False, reset=False)
            if self.defer_ir:  # I_k: reads buffer k's crops and T_k's C_pred (both graph-static)
                # its results go to buffers allocated outside the capture, each written by one
                # kernel: a graph-pool output could share memory with the graph's own scratch
                # (the feature distance's), which holds other bytes during a replay
                dev_ = step.last_C_pred.device
                ir_out = torch.zeros((), dtype=torch.float32, device=dev_)
                st = torch.zeros((step.last_C_pred.shape[0],), dtype=torch.int32, device=dev_)
                gi = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gi):
                    TrainStep.inlier_ratio_of(op, self.crops[k], step.last_C_pred, status=st, out=ir_out)
                self.logs[k]["IR"] = ir_out
                self.logs[k]["ir_index_status"] = st
                self.ir_graphs.append(gi)
            self.grads.append([p.grad for p in step.params])
            gb = None
            if self.split:
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb, pool=ga.pool()):
                    step.apply(allreduce=False, reset=False)
            self.train_a.append(ga)
            self.train_b.append(gb)
        self.formed = [torch.cuda.Event(), torch.cuda.Event()]   # C_k done
        self.consumed = [torch.cuda.Event(), torch.cuda.Event()]  # T_k done reading buffer k
        for k in range(2):
            self.consumed[k].record(self.main)
        self.i = 0
        self._form(0)

    def _replay_ir(self, k):
        """I_k on the side stream (after T_k released buffer k), then its completion event."""
        self.ir_graphs[k].replay()
        self.ir_done[k].record(self.side)
        self._ir_enqueued[k] = True

    def _form(self, k):
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.consumed[k])
            if self.defer_ir and self._trained[k]:  # the IR of the batch T_k last trained on
                self._replay_ir(k)
                self._trained[k] = False
            self.crop_graphs[k].replay()
            self.formed[k].record(self.side)

    def wait_ir(self, stream=None):
        """Order `stream` (default: the current stream) after every I_k enqueued so far, so the
        "IR" of every log returned before the last call is safe to read on it."""
        s = stream if stream is not None else torch.cuda.current_stream()
        for k in range(2):
            if self._ir_enqueued[k]:
                s.wait_event(self.ir_done[k])

    def flush(self, check: bool = True):
        """Compute the IR still pending for the last step (its buffer's I_k) and order the
        current stream after it: every log returned so far then holds its IR. check=True then
        reads the IR's per-crop index status of both buffers (a host sync: flush() runs outside
        timed loops) and raises PoseKernError if a point-map index was out of range."""
        if not self.defer_ir or self.i == 0:
            return
        cur = torch.cuda.current_stream()
        if cur != self.main:  # (as in __call__: the replay after the caller's queued work)
            self.main.wait_stream(cur)
        k = (self.i - 1) & 1
        if self._trained[k]:
            with torch.cuda.stream(self.side):
                self.side.wait_event(self.consumed[k])
                self._replay_ir(k)
            self._trained[k] = False
        self.wait_ir()
        if check:
            for log in self.logs:
                ops.check_index_status(log.get("ir_index_status"), "PipelinedTrainer IR (naive point map)")

    def __call__(self) -> dict:
        k = self.i & 1
        # a caller on another stream than the replays' (a private main stream, or a caller that
        # switched streams since construction): the step after the caller's queued work (its reads
        # of earlier logs / params), and the caller's stream after the step
        cur = torch.cuda.current_stream()
        if cur != self.main:
            self.main.wait_stream(cur)
        if not self.side_after:
            self._form(k ^ 1)                  # next batch's crops, concurrently
        with torch.cuda.stream(self.main):
            self.main.wait_event(self.formed[k])
            self.train_a[k].replay()
            if self.split:
                self.step.allreduce_grads(self.grads[k])
                self.train_b[k].replay()
            self.consumed[k].record(self.main)
        if self.side_after:
            self._form(k ^ 1)
        if cur != self.main:  # the caller's stream reads the step's outputs after it
            cur.wait_stream(self.main)
        self._trained[k] = True
        self.i += 1
        return self.logs[k]


class InferStep:
    """eval.py inference + test_RANSAC.py pose fit for a batch of crops."""

    def __init__(self, model: DPFMNet, hypotheses: int = 1024, seed: int = 0, max_dist: float = 0.05,
                 icp_evaluations: int = 0, icp_threshold: float = 0.2):
        """icp_evaluations > 0 refines each RANSAC pose by point-to-point ICP of the CAD against the
        observed crop (test_RANSAC.py:436-446 runs ICP after RANSAC, against the GT-posed CAD; the
        crop is the target available without ground truth), with that many evaluations enqueued
        (capturable: no host read) and the metrics also reported for the refined pose."""
        self.model, self.H, self.seed, self.max_dist = model, hypotheses, seed, max_dist
        self.icp_evaluations, self.icp_threshold = icp_evaluations, icp_threshold

    @torch.no_grad()
    def __call__(self, fb: FrameBatch, op: Operators, crops: Crops):
        return self.pose_stage(fb, op, crops, self.model_stage(fb, op, crops))

    @torch.no_grad()
    def model_stage(self, fb: FrameBatch, op: Operators, crops: Crops) -> dict:
        """DPFMNet forward and the naive solver's top-5 candidates (eval.py:80-87,
        spacial_filtering.py:32-38): the MFMA-bound first half of the step."""
        self.model.eval()
        C_pred, o12, o21, f1, f2, _, _ = self.model(model_batch(op, crops))
        B, V1, _ = op.cad_evecs.shape
        V2 = op.pc_evecs.shape[1]
        dev = C_pred.device
        # eval.py:85-87: the solver sees only the non-padding rows of each crop
        n1 = _counts(op.cad_n, B, V1, dev)
        n2 = _counts(crops.n2, B, V2, dev)
        top, _ = ops.feat_dist_topk(op.cad_evecs, C_pred, op.pc_evecs, n1, n2, 5)      # spacial_filtering.py:32-38
        cand = torch.stack([top.reshape(B, -1),
                            torch.arange(V2, device=dev)[None, :, None].expand(B, V2, 5).reshape(B, -1)], -1)
        return dict(C=C_pred, cand=cand, ncand=5 * n2)

    @torch.no_grad()
    def pose_stage(self, fb: FrameBatch, op: Operators, crops: Crops, m: dict) -> dict:
        """Rigidity filter, IR, RANSAC and the pose metrics (spacial_filtering.py:42-75,
        eval.py:89, test_RANSAC.py): the VALU-bound second half of the step."""
        C_pred, cand, ncand = m["C"], m["cand"], m["ncand"]
        B, V1, _ = op.cad_evecs.shape
        V2 = op.pc_evecs.shape[1]
        dev = C_pred.device
        rows, nsurv = ops.rigidity_filter(cand, ncand, op.cad_xyz, crops.pc32, op.rig_thr)  # :42-75
        p_pred = torch.gather(cand, 1, rows[..., None].expand(-1, -1, 2))                  # [B, L, 2]
        st_ir = torch.empty((B,), dtype=torch.int32, device=dev)
        st_rs = torch.empty((B,), dtype=torch.int32, device=dev)
        ir = ops.inlier_ratio(p_pred, nsurv, op.cad_xyz, crops.align32, op.ir_thr, layout=0, status=st_ir)  # eval.py:89
        # RANSAC on (CAD, crop in camera frame) with the surviving correspondences
        cor_off = torch.zeros(B + 1, dtype=torch.int64, device=dev)
        cor_off[1:] = torch.cumsum(nsurv.to(torch.int64), 0)
        L = p_pred.shape[1]
        ar = torch.arange(L, device=dev)[None]
        valid = ar < nsurv[:, None]
        # packed [sum n, 2] without reading the total on the host: crop b's i-th survivor goes
        # to row cor_off[b] + i of a B*L-row buffer (+1 spill row for the invalid slots)
        pos = torch.where(valid, cor_off[:-1, None] + ar, torch.full_like(ar, B * L)).reshape(-1)
        corres = torch.zeros((B * L + 1, 2), dtype=torch.int32, device=dev)
        corres.index_copy_(0, pos, p_pred.reshape(-1, 2).to(torch.int32))
        T, stats = ops.ransac(fb.cad64, fb.cad_off, crops.pc64, crops.off, corres, cor_off, self.H, seed=self.seed,
                              max_dist=self.max_dist, nmax=L, status=st_rs)
        T_gt = torch.zeros((B, 4, 4), dtype=torch.float64, device=dev)
        T_gt[:, :3, :3] = fb.R.view(B, 3, 3)
        T_gt[:, :3, 3] = fb.t
        T_gt[:, 3, 3] = 1.0
        # capacities of the packed point sets the pose stages read: the frame batch's CADs (fb.n1max, the
        # largest; the operator rows V1 may be a decimated CAD) and the crops (crops.ld)
        n1cap = max(int(fb.n1max or 0), V1)
        metrics = ops.pose_metrics(fb.cad64, fb.cad_off, n1cap, T, T_gt)
        # per crop 1: an index consumer (IR, RANSAC) met an out-of-range index (ops.check_index_status)
        out = dict(C=C_pred, cand=cand, p_pred=p_pred, n_corr=nsurv, ir=ir, T=T, ransac=stats, metrics=metrics,
                   corres=corres, cor_off=cor_off, index_status=st_ir | st_rs)
        if self.icp_evaluations > 0:
            T_icp, icp_stats = ops.icp_fixed(fb.cad64, fb.cad_off, crops.pc64, crops.off, T, self.icp_threshold,
                                             self.icp_evaluations, n1cap, max(int(crops.ld), V2))
            out.update(T_icp=T_icp, icp=icp_stats,
                       metrics_icp=ops.pose_metrics(fb.cad64, fb.cad_off, n1cap, T_icp, T_gt))
        return out


class GraphedInfer:
    """Crop formation + InferStep captured once into a HIP graph and replayed (the inference
    twin of GraphedTrainStep): frames, CAD models and operators stay resident; every replay
    re-forms the crops and re-runs the model, correspondence head, RANSAC and metrics. The
    returned dict's tensors are the graph's static outputs (overwritten by the next replay)."""

    def __init__(self, crop_formation: CropFormation, infer: InferStep, fb: FrameBatch, op: Operators,
                 warmup: int = 2):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                infer(fb, op, crop_formation(fb))
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = infer(fb, op, crop_formation(fb))

    def __call__(self) -> dict:
        self.graph.replay()
        return self.out


class PipelinedInfer:
    """Crop formation of batch i+1 overlapped with inference on batch i (the inference twin of
    PipelinedTrainer): graph C_k forms crops into buffer k on a side stream, graph I_k runs
    InferStep on buffer k on the main stream; events order C_k after I_k's previous use of the
    buffer and I_k after C_k. Crop formation (FPS, SOR: one workgroup per crop, latency-bound)
    then hides under the model, the correspondence head and RANSAC (wide kernels). Each call
    returns the static outputs of the graph it replayed (overwritten two calls later).

    stages=3 also splits InferStep at the candidates: M_k (model forward + top-5, MFMA-bound,
    many small launches) of batch i runs on the main stream while P_k (rigidity filter, IR,
    RANSAC, metrics: VALU-bound wide launches) of batch i-1 runs on a third stream, with three
    crop buffers (formation i+1, model i, pose i-1 in flight at once). Call i then returns the
    outputs of batch i-1 (None on the first call; flush() runs the last pending pose stage)."""

    def __init__(self, crop_formation: CropFormation, infer: InferStep, fb: FrameBatch, op: Operators,
                 warmup: int = 2, side_cus: int = 0, stages: int = 2):
        if stages not in (2, 3):
            raise ValueError("PipelinedInfer: stages must be 2 or 3")
        self.stages = stages
        self.main = torch.cuda.current_stream()
        self.side = torch.cuda.Stream()
        if side_cus > 0:  # disjoint CU sets for the two streams (cu_split_streams)
            self.main, self.side = cu_split_streams(side_cus)
            self.main.wait_stream(torch.cuda.current_stream())
        self.post = torch.cuda.Stream() if stages == 3 else self.main
        tmp = torch.cuda.Stream()
        tmp.wait_stream(self.main)
        with torch.cuda.stream(tmp):
            for _ in range(warmup):
                infer(fb, op, crop_formation(fb))
        self.main.wait_stream(tmp)
        torch.cuda.synchronize()
        nb = 2 if stages == 2 else 3
        self.nb = nb
        self.crop_graphs, self.crops, self.infer_graphs, self.outs = [], [], [], []
        self.pose_graphs, self.mids = [], []
        for k in range(nb):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):  # (InferStep reads no C_gt: none is solved here)
                self.crops.append(crop_formation(fb))
            self.crop_graphs.append(g)
        for k in range(nb):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                if stages == 2:
                    self.outs.append(infer(fb, op, self.crops[k]))
                else:
                    self.mids.append(infer.model_stage(fb, op, self.crops[k]))
            self.infer_graphs.append(g)
            if stages == 3:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    self.outs.append(infer.pose_stage(fb, op, self.crops[k], self.mids[k]))
                self.pose_graphs.append(g)
        self.formed = [torch.cuda.Event() for _ in range(nb)]
        self.modeled = [torch.cuda.Event() for _ in range(nb)]
        self.consumed = [torch.cuda.Event() for _ in range(nb)]  # buffer k's last reader done
        for k in range(nb):
            self.consumed[k].record(self.main)
        self.i = 0
        self._pending = None  # stages=3: the buffer whose pose stage is still to run
        self._form(0)

    def _form(self, k):
        with torch.cuda.stream(self.side):
            self.side.wait_event(self.consumed[k])
            self.crop_graphs[k].replay()
            self.formed[k].record(self.side)

    def _enter(self) -> torch.cuda.Stream:
        """The caller's stream; every stream that replays a graph writing returned outputs waits
        for it first, so the caller's reads of earlier outputs (enqueued before this call) finish
        before a replay overwrites them."""
        cur = torch.cuda.current_stream()
        for st in (self.main, self.post):
            if st != cur:
                st.wait_stream(cur)
        return cur

    @staticmethod
    def _hand_out(cur: torch.cuda.Stream, producer: torch.cuda.Stream, out):
        """Order the caller's stream after the graph that wrote `out` (no host sync)."""
        if out is not None and producer != cur:
            ev = torch.cuda.Event()
            ev.record(producer)
            cur.wait_event(ev)
        return out

    def _pose(self, k):
        with torch.cuda.stream(self.post):
            self.post.wait_event(self.modeled[k])
            self.pose_graphs[k].replay()
            self.consumed[k].record(self.post)
        return self.outs[k]

    def __call__(self):
        cur = self._enter()
        if self.stages == 2:
            k = self.i & 1
            self._form(k ^ 1)  # the next batch's crops, concurrently
            with torch.cuda.stream(self.main):
                self.main.wait_event(self.formed[k])
                self.infer_graphs[k].replay()
                self.consumed[k].record(self.main)
            self.i += 1
            return self._hand_out(cur, self.main, self.outs[k])
        k = self.i % 3
        self._form((self.i + 1) % 3)  # batch i+1 (its buffer's pose stage, batch i-2, is ordered before)
        with torch.cuda.stream(self.main):
            self.main.wait_event(self.formed[k])
            self.infer_graphs[k].replay()
            self.modeled[k].record(self.main)
        out = self._pose(self._pending) if self._pending is not None else None  # batch i-1
        self._pending = k
        self.i += 1
        return self._hand_out(cur, self.post, out)

    def flush(self):
        """stages=3: run the pose stage still pending (the last call's batch) and return its outputs."""
        if self.stages == 2 or self._pending is None:
            return None
        cur = self._enter()
        out = self._pose(self._pending)
        self._pending = None
        return self._hand_out(cur, self.post, out)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Rank-contiguous partition of n crops (configs[3]: 256 crops over 8 GPUs): rank r takes
    [r*n//world, (r+1)*n//world)."""
    return rank * n // world, (rank + 1) * n // world


def gather_results(local: dict, keys=("T", "ir", "n_corr", "metrics"), group: Optional[dist.ProcessGroup] = None,
                   world: int = 1) -> dict:
    """all_gather of the per-crop results of sharded inference (poses, IR, counts, metrics) so
    every rank holds the whole batch in global crop order. No collective runs with one rank.
    Shards may differ in size by one crop: padded to the largest, then trimmed."""
    if world <= 1:
        return {k: local[k] for k in keys}
    out = {}
    n = torch.tensor([local[keys[0]].shape[0]], device=local[keys[0]].device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    for k in keys:
        t = local[k]
        pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out[k] = torch.cat([p[:s] for p, s in zip(parts, sizes)], 0)
    return out
