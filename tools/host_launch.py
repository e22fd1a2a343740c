"""Host-side cost of replaying the training graphs (development aid): per call of the
overlapped trainer / the train-only step, the host time to enqueue vs the GPU time, and the
host time of one graph replay with and without a cross-stream event wait before it."""
import os, sys, time, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "6d-pose-estimation-for-unseen-categories_amd")]
import torch
import bench

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
sys.argv = [sys.argv[0]]
args = bench.parse()  # the bench's defaults (configs[1] training, crop formation overlapped)
tr, _, _, _, _ = bench.build_train(args, dev, 0, 1)
for _ in range(5):
    tr()
torch.cuda.synchronize()
n = 30
t0 = time.perf_counter()
for _ in range(n):
    tr()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"overlap: host enqueue {(t1 - t0) / n * 1e3:.3f} ms/step, wall {(t2 - t0) / n * 1e3:.3f} ms/step", flush=True)
main, side = tr.main, tr.side
ev = torch.cuda.Event()


def host_ms(fn, reps=10):
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    ts.sort()
    return f"median {ts[len(ts) // 2] * 1e3:.3f} ms, max {ts[-1] * 1e3:.3f} ms"


def replay_on(g, s, wait):
    def f():
        with torch.cuda.stream(s):
            if wait:
                ev.record(main if s is side else side)
                s.wait_event(ev)
            g.replay()
    return f


for name, g, s in (("crop graph (side)", tr.crop_graphs[0], side), ("train graph (main)", tr.train_a[0], main)):
    print(f"{name}: replay host {host_ms(replay_on(g, s, False))}; with a cross-stream wait first "
          f"{host_ms(replay_on(g, s, True))}", flush=True)
# replay while the other stream is busy with the other graph
def both():
    with torch.cuda.stream(main):
        tr.train_a[0].replay()
    a = time.perf_counter()
    with torch.cuda.stream(side):
        tr.crop_graphs[0].replay()
    return time.perf_counter() - a
torch.cuda.synchronize()
ts = sorted(both() for _ in range(10))
torch.cuda.synchronize()
print(f"crop graph replay host while the train graph runs: median {ts[5] * 1e3:.3f} ms", flush=True)

# GPU-side cost of the cross-stream events alone: the training graph replayed with the same
# wait / record pattern as the overlapped trainer, but no crop formation on the side stream
def events_only(n=30):
    torch.cuda.synchronize()
    a = time.perf_counter()
    for i in range(n):
        k = i & 1
        with torch.cuda.stream(side):
            side.wait_event(tr.consumed[k ^ 1])
            tr.formed[k ^ 1].record(side)
        main.wait_event(tr.formed[k])
        tr.train_a[k].replay()
        tr.consumed[k].record(main)
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3
def train_only(n=30):
    torch.cuda.synchronize()
    a = time.perf_counter()
    for i in range(n):
        tr.train_a[i & 1].replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3
def crop_only(n=30):
    torch.cuda.synchronize()
    a = time.perf_counter()
    with torch.cuda.stream(side):
        for i in range(n):
            tr.crop_graphs[i & 1].replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3
print(f"wall per step: train graphs alone {train_only():.3f} ms, with the event pattern {events_only():.3f} ms, "
      f"crop graphs alone {crop_only():.3f} ms", flush=True)

# the two graphs concurrently with no event coupling at all (T_k reads a buffer C_k may be
# rewriting: timing only): pure interference between the streams
def uncoupled(n=30):
    torch.cuda.synchronize()
    a = time.perf_counter()
    for i in range(n):
        k = i & 1
        with torch.cuda.stream(side):
            tr.crop_graphs[k ^ 1].replay()
        tr.train_a[k].replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3
def coupled_one_way(n=30):  # T waits for C, C never waits for T
    torch.cuda.synchronize()
    a = time.perf_counter()
    for i in range(n):
        k = i & 1
        with torch.cuda.stream(side):
            tr.crop_graphs[k ^ 1].replay()
            tr.formed[k ^ 1].record(side)
        main.wait_event(tr.formed[k])
        tr.train_a[k].replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - a) / n * 1e3
print(f"uncoupled streams {uncoupled():.3f} ms/step, T waits for C only {coupled_one_way():.3f} ms/step", flush=True)
