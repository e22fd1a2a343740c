"""Worker for test_distributed_gpu.py::test_rccl_flat_allreduce_world1: the training step's
gradient collective on RCCL (torch.distributed backend "nccl" = RCCL on ROCm) with one rank —
the only RCCL configuration a one-GPU box allows (RCCL rejects two ranks on one device). It
proves RCCL loads, initialises on the HIP allocator's memory and reduces TrainStep's flat
gradient buffer in place, in eager mode and between the two graphs of the split step
(scripts/train.py:121-124 + DDP's all-reduce)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import GraphedTrainStep, TrainStep, make_frame_batch
    torch.manual_seed(0)
    step = TrainStep(DPFMNet().to(dev), seed=0)
    assert step.flat_grads and step.world == 1
    # (1) the flat buffer: every .grad is a view; one RCCL all-reduce leaves it bit-equal
    fb, op = make_frame_batch(2, 256, 256, seed=5, device=dev)
    crops = CropFormation(n1=256, npoint=256, seed=1)(fb)
    step.forward_backward(op, crops)
    before = step.flat.detach().clone()
    assert float(before.abs().max()) > 0
    ptr = step.flat.data_ptr()
    step.allreduce_grads(force=True)
    torch.cuda.synchronize()
    assert step.flat.data_ptr() == ptr and torch.equal(step.flat, before), "RCCL all-reduce (world 1) changed the sum"
    for p, v in zip(step.params, step.gviews):
        assert p.grad.data_ptr() == v.data_ptr(), "a .grad is not a view of the flat buffer"
    # a known pattern through the same buffer: the collective reads and writes the views
    step.flat.copy_(torch.arange(step.flat.numel(), dtype=torch.float32, device=dev))
    dist.all_reduce(step.flat)
    torch.cuda.synchronize()
    assert torch.equal(step.params[3].grad.reshape(-1), step.gviews[3].reshape(-1))
    off = sum(p.numel() for p in step.params[:3])
    exp = torch.arange(off, off + step.params[3].numel(), dtype=torch.float32, device=dev)
    assert torch.equal(step.params[3].grad.reshape(-1), exp)
    step.apply(allreduce=False)
    # (2) the split graphed step (graph A | RCCL all-reduce | graph B), forced at world 1
    torch.manual_seed(1)
    gstep = TrainStep(DPFMNet().to(dev), seed=0, capturable=True)
    g = GraphedTrainStep(CropFormation(n1=256, npoint=256, seed=1), gstep, fb, op, warmup=1)
    for _ in range(2):
        g.graph_a.replay()
        ref = gstep.flat.detach().clone()
        gstep.allreduce_grads(force=True)
        torch.cuda.synchronize()
        assert torch.equal(gstep.flat, ref)
    dist.barrier()
    dist.destroy_process_group()
    print("rccl ok", flush=True)


if __name__ == "__main__":
    main()
