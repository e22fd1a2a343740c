"""What HBM bandwidth can a launch of a given size reach on this box? torch's copy (read +
write) and sum (read) over 4 MB - 1 GB buffers, graph-replayed (20 launches back to back),
next to the per-point layer 128->64 at R = 65536 (50 MB moved). Calibrates the layer
roofline: a 50 MB launch cannot reach the 8 TB/s peak when copies of that size do not."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch  # noqa: E402


def timed(f, n=20):
    f()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
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
    return e0.elapsed_time(e1) * 1e3 / n


dev = torch.device("cuda:0")
for mb in (4, 8, 17, 33, 67, 134, 268, 1074):
    n = mb * (1 << 20) // 4
    # rotate over several buffers so a launch's input is not the previous launch's output
    src = [torch.randn(n, device=dev) for _ in range(4 if mb <= 268 else 1)]
    dst = torch.empty(n, device=dev)
    out = torch.empty((), device=dev)
    k = [0]

    def cp():
        dst.copy_(src[k[0] % len(src)])
        k[0] += 1

    def sm():
        torch.sum(src[k[0] % len(src)], dim=(0,), out=out)
        k[0] += 1
    tc, ts = timed(cp), timed(sm)
    print(f"{mb:5d} MB: copy {tc:8.2f} us {2 * n * 4 / tc / 1e3:6.0f} GB/s   sum {ts:8.2f} us {n * 4 / ts / 1e3:6.0f} GB/s",
          flush=True)
    del src, dst
