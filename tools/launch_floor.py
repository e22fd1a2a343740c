"""Device time per launch of back-to-back tiny kernels replayed from a HIP graph: the
per-kernel floor a graph-replayed step pays for every launch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
from dpfm_amd import ops

dev = torch.device("cuda:0")
t = torch.zeros(64, device=dev)
x = torch.randn(64, 32, device=dev)
w = torch.randn(32, 32, device=dev)
cases = {"torch add_ (64 floats)": lambda: t.add_(1.0),
         "pk_linear_fwd (64 x 32 -> 32)": lambda: ops.linear_fwd(x, w, None, channels_first=False)}
for name, f in cases.items():
    for n in (50, 200):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    f()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        print(f"{name}: {n} launches in a graph: {e0.elapsed_time(e1) * 1e3 / n:.2f} us per launch "
              f"(DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')})", flush=True)
