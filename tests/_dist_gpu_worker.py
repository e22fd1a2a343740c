"""Worker for test_distributed_gpu.py (launched by torch.distributed.run, 2 ranks sharing
cuda:0, gloo): TrainStep's flat-gradient all-reduce on HIP tensors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import TrainStep, make_frame_batch
    torch.manual_seed(0)
    model = DPFMNet().to(dev)
    step = TrainStep(model, seed=rank)
    assert step.flat_grads and step.world == world
    # (1) the gradients are views of one flat buffer: one collective gives the mean
    for p, v in zip(step.params, step.gviews):
        p.grad = v
    step.flat.fill_(float(rank + 1))
    step.allreduce_grads()
    torch.cuda.synchronize()
    exp = sum(range(1, world + 1)) / world
    assert all(bool((p.grad == exp).all()) for p in step.params), "flat all-reduce mean"
    # (2) a real step on each rank's own crops: parameters stay identical across ranks
    fb, op = make_frame_batch(2, 256, 256, seed=100 * rank, device=dev)
    crops = CropFormation(n1=256, npoint=256, seed=rank)(fb)
    step(op, crops)
    torch.cuda.synchronize()
    flat_p = torch.cat([p.detach().reshape(-1) for p in step.params]).cpu()
    out = [torch.zeros_like(flat_p) for _ in range(world)]
    dist.all_gather(out, flat_p)
    assert all(torch.equal(out[0], o) for o in out), "parameters diverged across ranks"
    # (3) the HIP-graph paths bench.py uses for N > 1: graph A (crops -> backward), the eager
    # flat all-reduce, graph B (clip + RMSprop)
    from dpfm_amd.pipeline import GraphedTrainStep, PipelinedTrainer

    def same_params(st):
        flat = torch.cat([p.detach().reshape(-1) for p in st.params]).cpu()
        got = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(got, flat)
        return all(torch.equal(got[0], o) for o in got)

    cf = CropFormation(n1=256, npoint=256, seed=rank)
    torch.manual_seed(1)
    gstep = TrainStep(DPFMNet().to(dev), seed=rank, capturable=True)
    g = GraphedTrainStep(cf, gstep, fb, op, warmup=1)
    assert g.split
    for _ in range(3):
        g.graph_a.replay()                       # this rank's gradient into the flat buffer
        local = gstep.flat.detach().clone().cpu()
        every = [torch.zeros_like(local) for _ in range(world)]
        dist.all_gather(every, local)
        gstep.allreduce_grads()
        torch.cuda.synchronize()
        mean = torch.stack(every).mean(0)
        assert torch.allclose(gstep.flat.cpu(), mean, rtol=1e-6, atol=1e-7 * float(mean.abs().max())), \
            "graphed step: averaged gradient != mean of the ranks' gradients"
        g.graph_b.replay()
        torch.cuda.synchronize()
        assert same_params(gstep), "graphed step: parameters diverged across ranks"
    torch.manual_seed(2)
    pstep = TrainStep(DPFMNet().to(dev), seed=rank, capturable=True)
    pipe = PipelinedTrainer(cf, pstep, fb, op, warmup=1)
    for _ in range(4):
        pipe()
        torch.cuda.synchronize()
        assert same_params(pstep), "pipelined trainer: parameters diverged across ranks"
        flat = pstep.flat.detach().cpu()
        got = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(got, flat)
        assert all(torch.equal(got[0], o) for o in got), "pipelined trainer: reduced gradients differ"
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("dist-gpu ok", flush=True)


if __name__ == "__main__":
    main()
