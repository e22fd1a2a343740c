"""GPU: the batched device pipeline (crop formation -> train step / inference + pose)
runs sync-free and agrees with the per-crop oracle chain."""
import numpy as np
import pytest
import torch

from oracle import dpfm_oracle as O

pytestmark = pytest.mark.gpu


def test_crop_formation_chain_matches_oracle(device, coracle):
    from _util import c_fps
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.dataset.synthetic import make_frame, cad_points
    from dpfm_amd.pipeline import make_frame_batch
    F, N = 4, 1024
    fb, op = make_frame_batch(F, N, N, seed=50, device=device)
    crops = CropFormation(n1=N, npoint=N, seed=3)(fb)
    torch.cuda.synchronize()
    start = None
    pc64 = crops.pc64.cpu().numpy()
    al = crops.align64.cpu().numpy()
    pairs = crops.pairs.cpu().numpy()
    npairs = crops.npairs.cpu().numpy()
    for f in range(F):
        fr = make_frame(50 + f)
        pcd = O.remove_outliers(O.dpt_2_pcld(fr.depth, 1000 / fr.depth_scale, fr.K, fr.mask == 255))
        from dpfm_amd import ops
        # start index of crop f: splitmix hash of (seed, f) as documented in posekern.h
        pol = ops.fps_npoint(ops.packed_offsets([pcd.shape[0]] * F, device), fixed=N, seed=3)
        st = int(pol["start"][f])
        idx = c_fps(coracle, pcd.astype(np.float32), st, N)
        sel = pcd[idx]
        np.testing.assert_array_equal(pc64[f * N:(f + 1) * N], sel)
        align = O.transform(sel, fr.R_m2c, fr.t_m2c, inv=True)
        np.testing.assert_array_equal(al[f * N:(f + 1) * N], align)
        cad = cad_points(fr, N, 50 + f)
        P = O.find_positives(cad, align, r=0.05 * fr.diam_cad)
        assert npairs[f] == P.shape[0]
        np.testing.assert_array_equal(pairs[f, :npairs[f]], P)


def test_train_and_infer_steps(device):
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, InferStep, make_frame_batch
    torch.manual_seed(0)
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=70, device=device)
    crops = CropFormation(n1=N, npoint=N)(fb)
    model = DPFMNet().to(device)
    step = TrainStep(model)
    w0 = [p.detach().clone() for p in model.parameters()]
    log = step(op, crops)
    torch.cuda.synchronize()
    assert torch.isfinite(log["loss"]) and 0.0 <= float(log["IR"]) <= 1.0
    assert any(not torch.equal(a, b.detach()) for a, b in zip(w0, model.parameters()))
    out = InferStep(model, hypotheses=256)(fb, op, crops)
    torch.cuda.synchronize()
    assert out["T"].shape == (F, 4, 4) and torch.isfinite(out["metrics"]).all()


def test_grouped_wgrad_step_matches_serial(device):
    """TrainStep's grouped weight gradients (layers.GroupedWgrad: every per-point layer's
    dW / db recorded during backward, computed in one pk_linear_wgrad_grouped launch pair,
    shared layers accumulating). The recorded (x, dy) of every call are checked against an
    fp64 recomputation within the fp32 summation bound 1e-5 * sum_r |dy||x|; every layer
    parameter is fed; the per-layer autograd path agrees within 2x that bound plus its own
    run-to-run spread (torch ops without deterministic kernels)."""
    from dpfm_amd import layers
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, make_frame_batch
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=90, device=device)
    crops = CropFormation(n1=N, npoint=N)(fb)
    models = []
    for _ in range(3):
        torch.manual_seed(3)
        models.append(DPFMNet().to(device))
    steps = [TrainStep(models[0], seed=2, grouped=False), TrainStep(models[1], seed=2, grouped=False),
             TrainStep(models[2], seed=2, grouped=True)]
    assert steps[2].side is not None and len(steps[2].side.params) > 30 and steps[0].side is None
    rec = []
    orig = layers.ops.linear_wgrad_grouped

    def spy(calls):
        rec.extend((c[0].detach().clone(), c[1].detach().clone(), c[2], c[3], c[4], c[5]) for c in calls)
        return orig(calls)

    layers.ops.linear_wgrad_grouped = spy
    try:
        for s in steps:
            s.forward_backward(op, crops)
    finally:
        layers.ops.linear_wgrad_grouped = orig
    torch.cuda.synchronize()
    # fp64 truth and bound per output buffer from the recorded calls
    truth = {}
    for x, dy, cf, dw, db, acc in rec:
        if cf:
            X, D = x.transpose(1, 2).reshape(-1, x.shape[1]).double(), dy.transpose(1, 2).reshape(-1, dy.shape[1]).double()
        else:
            X, D = x.reshape(-1, x.shape[-1]).double(), dy.reshape(-1, dy.shape[-1]).double()
        key = dw.data_ptr()
        assert acc == (key in truth)
        t = (D.t() @ X, D.abs().t() @ X.abs(), D.sum(0), D.abs().sum(0), dw, db)
        if key in truth:
            u = truth[key]
            t = (u[0] + t[0], u[1] + t[1], u[2] + t[2], u[3] + t[3], dw, db)
        truth[key] = t
    n_params = n_direct = 0
    for (n, p0), p1, p2 in zip(models[0].named_parameters(), models[1].parameters(), models[2].parameters()):
        g0, g1, g2 = p0.grad, p1.grad, p2.grad
        assert g2 is not None, n
        hit = [t for t in truth.values() if t[4].data_ptr() == g2.data_ptr() or
               (t[5] is not None and t[5].data_ptr() == g2.data_ptr())]
        if not hit:  # not a per-point layer parameter (diffusion_time): written whole by the kernel
            assert n.endswith("diffusion_time"), n  # (GroupedWgrad.direct), equal to the serial step's
            assert (g2 - g1).abs().max().item() <= 1e-5 * g1.abs().max().item(), n
            n_direct += 1
            continue
        n_params += 1
        w, bw, b, bb, dw, db = hit[0]
        is_w = dw.data_ptr() == g2.data_ptr()
        ref, bound = (w, bw) if is_w else (b, bb)
        ref, bound = ref.reshape(g2.shape), bound.reshape(g2.shape)
        assert (g2.double() - ref).abs().le(1e-5 * bound + 1e-30).all(), n
        spread = (g0 - g1).abs().max().item()
        assert (g0.double() - g2.double()).abs().le(2e-5 * bound + 4 * spread + 1e-30).all(), (n, spread)
    assert n_params == len(steps[2].side.params) and n_direct == len(steps[2].side.direct_params)


def test_grouped_wgrad_keeps_diffusion_time_grads_on_module_path(device, monkeypatch):
    """On the per-module encoder path (FUSED_ENCODER = False) no kernel writes the diffusion-time
    gradients whole (GroupedWgrad.direct is never called): autograd accumulates them into the
    grouped step's .grad buffers, which end() must leave alone. Grouped and serial steps agree on
    them (within fp32 spread) over two consecutive backwards, and they are nonzero."""
    from dpfm_amd import diffusion_net as DN
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, make_frame_batch
    monkeypatch.setattr(DN, "FUSED_ENCODER", False)
    F, N = 2, 256
    fb, op = make_frame_batch(F, N, N, seed=93, device=device)
    crops = CropFormation(n1=N, npoint=N)(fb)
    models = []
    for _ in range(2):
        torch.manual_seed(4)
        models.append(DPFMNet().to(device))
    serial, grouped = TrainStep(models[0], seed=3, grouped=False), TrainStep(models[1], seed=3, grouped=True)
    assert grouped.side is not None and len(grouped.side.direct_params) > 0
    for _ in range(2):  # the second backward must not add onto the first one's values
        for s in (serial, grouped):
            s.forward_backward(op, crops)
        torch.cuda.synchronize()
        n = 0
        for (name, p0), p1 in zip(models[0].named_parameters(), models[1].parameters()):
            if not name.endswith("diffusion_time"):
                continue
            g0, g1 = p0.grad, p1.grad
            assert g1 is not None and float(g1.abs().max()) > 0, name
            assert (g1 - g0).abs().max().item() <= 1e-5 * g0.abs().max().item(), name
            n += 1
        assert n == len(grouped.side.direct_params)
        for s in (serial, grouped):
            s.opt.zero_grad(set_to_none=True)


def test_graphed_train_step_matches_eager(device):
    """The HIP-graph replay of crop formation + training step (GraphedTrainStep) follows
    the same trajectory as the eager step from the same state (same RNG stream)."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedTrainStep, TrainStep, make_frame_batch
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=90, device=device)
    cf = CropFormation(n1=N, npoint=N, seed=1)
    torch.manual_seed(0)
    m_eager = DPFMNet().to(device)
    m_graph = DPFMNet().to(device)
    m_graph.load_state_dict(m_eager.state_dict())
    eager = TrainStep(m_eager, seed=5, capturable=True)
    graph_step = TrainStep(m_graph, seed=5, capturable=True)
    g = GraphedTrainStep(cf, graph_step, fb, op, warmup=2)   # 2 eager warm-up steps + capture
    for _ in range(2):                                         # same 2 warm-up steps on the twin
        eager(op, cf(fb))
    # the step is deterministic (NCE gradients summed in slot order, grouped weight gradients
    # by fixed trees, no float atomics): from a common state (the twin is re-synced to the
    # graph's parameters, optimizer state and NCE draw counter before every step) the replay
    # and the eager step agree bit for bit
    for _ in range(3):
        eager.load_state_from(graph_step)
        le = {k: v.clone() for k, v in eager(op, cf(fb)).items()}
        lg = {k: v.clone() for k, v in g().items()}
        torch.cuda.synchronize()
        for k in ("loss", "IR"):
            assert torch.equal(le[k], lg[k]), (k, le[k], lg[k])
        diff = [n for (n, a), b in zip(m_eager.named_parameters(), m_graph.parameters()) if not torch.equal(a, b)]
        assert not diff, diff


def test_pipelined_trainer_matches_eager(device):
    """PipelinedTrainer (crop formation of batch i+1 on a second stream, ping-pong crop
    buffers, every piece a graph replay) follows the eager trajectory: the crops of a
    static frame batch are identical every step, so the loss sequence must agree."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import PipelinedTrainer, TrainStep, make_frame_batch
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=91, device=device)
    cf = CropFormation(n1=N, npoint=N, seed=2)
    torch.manual_seed(0)
    m_eager, m_pipe = DPFMNet().to(device), DPFMNet().to(device)
    m_pipe.load_state_dict(m_eager.state_dict())
    eager, ps = TrainStep(m_eager, seed=7, capturable=True), TrainStep(m_pipe, seed=7, capturable=True)
    pipe = PipelinedTrainer(cf, ps, fb, op, warmup=2)
    for _ in range(2):
        eager(op, cf(fb))
    for _ in range(4):  # step by step from a common state (see the graphed-step test): bit for bit
        eager.load_state_from(ps)
        le = eager(op, cf(fb))
        lp = pipe()
        pipe.flush()  # the step's IR, computed beside the training stream (PipelinedTrainer doc)
        torch.cuda.synchronize()
        assert torch.equal(le["loss"], lp["loss"]), (le["loss"], lp["loss"])
        assert torch.equal(le["IR"], lp["IR"]), (le["IR"], lp["IR"])
        diff = [n for (n, a), b in zip(m_eager.named_parameters(), m_pipe.parameters()) if not torch.equal(a, b)]
        assert not diff, diff


def test_pipelined_trainer_private_stream_ordered_with_caller(device):
    """PipelinedTrainer driven from a caller stream other than its replay stream — its default
    main stream, or a private one (main_priority=1): every call waits for the caller's
    queued work and hands the step back to the caller's stream, so copies of the loss taken on the
    caller stream right after each call, with no device synchronisation, are the step's losses and
    agree between the two pipelines step for step (same seeds, same crops); flush() checks the
    IR's index status (clean crops: no error)."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import PipelinedTrainer, TrainStep, make_frame_batch
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=93, device=device)
    torch.manual_seed(2)
    ma, mb = DPFMNet().to(device), DPFMNet().to(device)
    mb.load_state_dict(ma.state_dict())
    losses = []
    for m, prio in ((ma, 0), (mb, 1)):
        torch.manual_seed(3)  # (the same global RNG state for both pipelines' warm-up and capture)
        p = PipelinedTrainer(CropFormation(n1=N, npoint=N, seed=5), TrainStep(m, seed=9, capturable=True), fb, op,
                             warmup=2, main_priority=prio)
        caller = torch.cuda.Stream()
        got = []
        with torch.cuda.stream(caller):
            for _ in range(4):
                got.append(p()["loss"].clone())
            p.flush()
        torch.cuda.synchronize()
        losses.append(got)
    for a, b in zip(*losses):
        assert torch.equal(a, b), (a, b)
    assert all(float(a) > 0.0 for a in losses[0])  # (real losses, not a copy taken before the step)


def test_pipelined_trainer_deferred_ir_readers(device):
    """The deferred IR is written by a side-stream graph: wait_ir() orders the reader after
    every I_k enqueued so far (the logs of all calls but the last), flush() computes the last
    one (test_pipelined_trainer_matches_eager checks the values against the eager step)."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import PipelinedTrainer, TrainStep, make_frame_batch
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=92, device=device)
    cf = CropFormation(n1=N, npoint=N, seed=3)
    torch.manual_seed(1)
    ps = TrainStep(DPFMNet().to(device), seed=8, capturable=True)
    pipe = PipelinedTrainer(cf, ps, fb, op, warmup=1)
    logs = [pipe() for _ in range(3)]
    pipe.wait_ir()
    early = [logs[0]["IR"].clone(), logs[1]["IR"].clone()]  # calls 0 and 1 (I_0, I_1 enqueued)
    pipe.flush()
    last = logs[2]["IR"].clone()
    torch.cuda.synchronize()
    for ir in early + [last]:
        assert 0.0 <= float(ir) <= 1.0
    # call 1's IR read after wait_ir() is final (nothing writes buffer 1's slot again before call 3)
    assert torch.equal(early[1], logs[1]["IR"])
    assert torch.equal(last, logs[2]["IR"])


@pytest.mark.parametrize("scale", [10.0, 1e-3])
def test_fused_clip_rmsprop_matches_torch(device, scale):
    """pk_clip_rmsprop (TrainStep.apply's clip_grad_norm_(5.0) + RMSprop(5e-4) in one launch)
    vs torch's clip_grad_norm_ + RMSprop.step over three steps with fresh gradients each
    step, clipping active (scale 10) and inactive (1e-3): parameters, clipped gradients and
    square_avg within fp32 rounding (2e-6 relative to each tensor's scale)."""
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep
    torch.manual_seed(4)
    ma, mb = DPFMNet().to(device), DPFMNet().to(device)
    mb.load_state_dict(ma.state_dict())
    sa, sb = TrainStep(ma, fused_opt=True), TrainStep(mb, fused_opt=False)
    assert sa.fused_opt and not sb.fused_opt
    g = torch.Generator(device=device).manual_seed(1)
    for it in range(3):
        for p, q in zip(ma.parameters(), mb.parameters()):
            gr = torch.randn(p.shape, device=device, generator=g) * scale
            p.grad, q.grad = gr.clone(), gr.clone()
        ga = [p.grad for p in ma.parameters()]
        gb = [q.grad for q in mb.parameters()]
        sa.apply(reset=False)
        sb.apply(reset=False)
        torch.cuda.synchronize()
        for (n, p), q, x, y in zip(ma.named_parameters(), mb.parameters(), ga, gb):
            tol = 2e-6 * max(float(q.detach().abs().max()), 1e-30)
            assert (p.detach() - q.detach()).abs().max().item() <= tol, (it, n)
            assert (x - y).abs().max().item() <= 2e-6 * float(y.abs().max()) + 1e-30, (it, n)
            sqa, sqb = sa.opt.state[p]["square_avg"], sb.opt.state[q]["square_avg"]
            assert (sqa - sqb).abs().max().item() <= 2e-6 * float(sqb.abs().max()) + 1e-30, (it, n)
        assert float(sa.opt.state[next(ma.parameters())]["step"]) == it + 1


def test_pipelined_infer_matches_graphed(device):
    """PipelinedInfer (crop formation of the next batch on a side stream, two ping-pong buffers)
    returns, call after call, exactly what the single-stream GraphedInfer returns on the same
    resident frames."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedInfer, InferStep, PipelinedInfer, make_frame_batch
    torch.manual_seed(0)
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=71, device=device)
    model = DPFMNet().to(device).eval()
    g = GraphedInfer(CropFormation(n1=N, npoint=N, seed=3), InferStep(model, hypotheses=256), fb, op)
    ref = {k: v.clone() for k, v in g().items() if torch.is_tensor(v)}
    p = PipelinedInfer(CropFormation(n1=N, npoint=N, seed=3), InferStep(model, hypotheses=256), fb, op)
    for _ in range(4):
        out = p()
        torch.cuda.synchronize()
        for key in ("T", "ir", "n_corr", "metrics", "p_pred"):
            assert torch.equal(out[key], ref[key]), key


def test_three_stage_pipelined_infer_matches_graphed(device):
    """PipelinedInfer(stages=3): crop formation (side stream), model + top-5 (main) and rigidity /
    IR / RANSAC / metrics (third stream) of three consecutive batches in flight; every batch's
    outputs equal the single-stream GraphedInfer's, one call late, and flush() returns the last."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedInfer, InferStep, PipelinedInfer, make_frame_batch
    torch.manual_seed(0)
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=71, device=device)
    model = DPFMNet().to(device).eval()
    g = GraphedInfer(CropFormation(n1=N, npoint=N, seed=3), InferStep(model, hypotheses=256), fb, op)
    ref = {k: v.clone() for k, v in g().items() if torch.is_tensor(v)}
    p = PipelinedInfer(CropFormation(n1=N, npoint=N, seed=3), InferStep(model, hypotheses=256), fb, op, stages=3)
    assert p() is None
    outs = [p() for _ in range(5)] + [p.flush()]
    torch.cuda.synchronize()
    for out in outs[-3:]:  # (the static outputs of the three pose graphs)
        for key in ("T", "ir", "n_corr", "metrics", "p_pred", "C"):
            assert torch.equal(out[key], ref[key]), key


def test_pipelined_infer_outputs_ordered_on_caller_stream(device):
    """PipelinedInfer hands its outputs to the caller's current stream: copies taken
    on that stream right after each call, with no device synchronisation in between, equal the
    single-stream graph's outputs — for stages=3 (pose graphs on a private stream) and from a
    caller stream other than the pipeline's main stream."""
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedInfer, InferStep, PipelinedInfer, make_frame_batch
    torch.manual_seed(0)
    F, N = 4, 512
    fb, op = make_frame_batch(F, N, N, seed=73, device=device)
    model = DPFMNet().to(device).eval()
    g = GraphedInfer(CropFormation(n1=N, npoint=N, seed=4), InferStep(model, hypotheses=256), fb, op)
    ref = {k: v.clone() for k, v in g().items() if torch.is_tensor(v)}
    torch.cuda.synchronize()
    for stages in (3, 2):
        p = PipelinedInfer(CropFormation(n1=N, npoint=N, seed=4), InferStep(model, hypotheses=256), fb, op,
                           stages=stages)
        caller = torch.cuda.Stream()
        copies = []
        with torch.cuda.stream(caller):
            for _ in range(6):
                out = p()
                if out is not None:
                    copies.append({k: out[k].clone() for k in ("T", "ir", "metrics", "C")})
            if stages == 3:
                out = p.flush()
                copies.append({k: out[k].clone() for k in ("T", "ir", "metrics", "C")})
        torch.cuda.synchronize()
        assert len(copies) == 6
        for c in copies:
            for key, v in c.items():
                assert torch.equal(v, ref[key]), (stages, key)


def test_infer_step_with_icp_matches_standalone_icp(device):
    """InferStep(icp_evaluations=E) refines the RANSAC poses against the crops exactly as the
    host-polled ops.icp with max_iteration E - 1 does, and stays HIP-graph capturable."""
    from dpfm_amd import ops
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedInfer, InferStep, make_frame_batch
    torch.manual_seed(0)
    F, N, E = 4, 512, 12
    fb, op = make_frame_batch(F, N, N, seed=72, device=device)
    model = DPFMNet().to(device).eval()
    crops = CropFormation(n1=N, npoint=N, seed=2)(fb)
    out = InferStep(model, hypotheses=256, icp_evaluations=E)(fb, op, crops)
    T, st = ops.icp(fb.cad64, fb.cad_off, crops.pc64, crops.off, out["T"], 0.2, E - 1, nsrc_max=N, ntgt_max=N)
    assert torch.equal(out["T_icp"], T) and torch.equal(out["icp"], st)
    g = GraphedInfer(CropFormation(n1=N, npoint=N, seed=2), InferStep(model, hypotheses=256, icp_evaluations=E), fb, op)
    o2 = g()
    torch.cuda.synchronize()
    assert torch.equal(o2["T_icp"], out["T_icp"]) and torch.isfinite(o2["metrics_icp"]).all()
