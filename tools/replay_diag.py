"""Dev diagnostic: eager vs HIP-graph replays of the training step over several steps
(tests/test_pipeline_gpu.py::test_graphed_train_step_matches_eager, with per-step prints).

  python tools/replay_diag.py [cublas|cublaslt|default] [graph|pipe]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] in ("cublas", "cublaslt"):
    torch.backends.cuda.preferred_blas_library(sys.argv[1])
mode = sys.argv[2] if len(sys.argv) > 2 else "graph"
print("blas:", torch.backends.cuda.preferred_blas_library(), "mode:", mode, flush=True)

from dpfm_amd.dataset.object import CropFormation  # noqa: E402
from dpfm_amd.models.dpfm import DPFMNet  # noqa: E402
from dpfm_amd.pipeline import GraphedTrainStep, TrainStep, make_frame_batch  # noqa: E402

dev = torch.device("cuda:0")
F_, N = 4, 512
fb, op = make_frame_batch(F_, N, N, seed=90, device=dev)
cf = CropFormation(n1=N, npoint=N, seed=1)
torch.manual_seed(0)
m_e, m_g = DPFMNet().to(dev), DPFMNet().to(dev)
m_g.load_state_dict(m_e.state_dict())
eager, gs = TrainStep(m_e, seed=5, capturable=True), TrainStep(m_g, seed=5, capturable=True)
g = GraphedTrainStep(cf, gs, fb, op, warmup=2)
for _ in range(2):
    eager(op, cf(fb))
for i in range(5):
    le = {k: float(v) for k, v in eager(op, cf(fb)).items()}
    lg = {k: float(v) for k, v in g().items()}
    pe = torch.cat([p.detach().flatten() for p in m_e.parameters()])
    pg = torch.cat([p.detach().flatten() for p in m_g.parameters()])
    print(f"step {i}: eager loss {le['loss']:.6f} IR {le['IR']:.5f} | graph loss {lg['loss']:.6f} IR {lg['IR']:.5f} "
          f"| params max|diff| {float((pe - pg).abs().max()):.3e} finite(graph) {bool(torch.isfinite(pg).all())}",
          flush=True)
