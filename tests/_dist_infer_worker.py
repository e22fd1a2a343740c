"""Worker for test_distributed_gpu.py::test_sharded_inference (torch.distributed.run, 2 ranks
sharing cuda:0, gloo): configs[3]-style batch-sharded inference. Rank r forms and infers
the crops [r*G/2, (r+1)*G/2) of a G-crop batch (no collective on the data path), the
per-crop results are all_gathered, and rank 0 checks them bit for bit against one process
running the whole batch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

G, N, BASE = 4, 512, 500


def run(lo, hi, dev):
    from dpfm_amd.dataset.object import CropFormation
    from dpfm_amd.models.dpfm import DPFMNet
    from dpfm_amd.pipeline import InferStep, make_frame_batch
    fb, op = make_frame_batch(hi - lo, N, N, seed=BASE + lo, device=dev)
    crops = CropFormation(n1=N, npoint=N, seed=3, base=lo)(fb)
    torch.manual_seed(0)
    model = DPFMNet().to(dev)
    return InferStep(model, hypotheses=256, seed=1)(fb, op, crops)


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    from dpfm_amd.pipeline import gather_results, shard_range
    lo, hi = shard_range(G, rank, world)
    local = run(lo, hi, dev)
    keys = ("T", "ir", "n_corr", "metrics", "C")
    mine = gather_results({k: local[k].cpu() for k in keys}, keys=keys, world=world)
    if rank == 0:
        full = run(0, G, dev)
        for k in keys:
            a, b = mine[k], full[k].cpu()
            assert a.shape == b.shape and torch.equal(a, b), (k, (a.double() - b.double()).abs().max())
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        print("sharded-infer ok", flush=True)


if __name__ == "__main__":
    main()
