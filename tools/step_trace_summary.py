"""Summarise a rocprofv3 kernel trace of bench.py's replayed steps: busy time per queue,
idle gaps, and the top kernels by total time over the last 10 steps' window."""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the timed window: the last `steps` steps (bench.py's ms_per_step from its JSON line)
import json, re
bench = next(json.loads(l) for l in reversed(open(sys.argv[2]).read().splitlines()) if l.startswith('{"metric"'))
steps = int(bench["steps"])
t1 = max(int(r["End_Timestamp"]) for r in rows)
lo = t1 - int(steps * bench["ms_per_step"] * 1e6)
print(f"ms_per_step {bench['ms_per_step']} x {steps}")
win = [r for r in rows if int(r["Start_Timestamp"]) >= lo]
span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6
byq = collections.defaultdict(list)
for r in win:
    byq[r.get("Queue_Id", r.get("Stream_Id", "?"))].append(r)
print(f"window {span:.3f} ms, {len(win)} kernels ({len(win)/steps:.0f} per step)")
for q, rs in byq.items():
    busy = 0
    end = None
    gaps = []
    for r in rs:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and s > end:
            gaps.append(s - end)
        busy += e - s
        end = max(end or 0, e)
    print(f"queue {q}: {len(rs)/steps:.0f} kernels/step, busy {busy/1e6/steps:.3f} ms/step, gaps {sum(gaps)/1e6/steps:.3f} ms/step, "
          f"mean gap {sum(gaps)/max(len(gaps),1)/1e3:.2f} us")
tot = collections.defaultdict(lambda: [0, 0])
for r in win:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("at::native"):  # keep the functor: which elementwise op
        m = re.findall(r"at::native::(?:\(anonymous namespace\)::)?([A-Za-z_]+(?:Functor[A-Za-z_]*)?|[a-z_]+_kernel[a-z_]*)", r["Kernel_Name"])
        n = "/".join(dict.fromkeys(m[:4]))[:110]
    else:
        n = re.split(r"[(<]", n)[0][:90]
    tot[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot[n][1] += 1
for n, (t, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:int(sys.argv[3]) if len(sys.argv) > 3 else 45]:
    print(f"{t/1e3/steps:8.1f} us/step {c/steps:6.1f}/step  {n}")

# the main queue's kernels of the last step, in issue order (duration, gap before it)
def short(r):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("at::native"):
        m = re.findall(r"at::native::(?:\(anonymous namespace\)::)?([A-Za-z_]+(?:Functor[A-Za-z_]*)?|[a-z_]+_kernel[a-z_]*)", r["Kernel_Name"])
        return "/".join(dict.fromkeys(m[:4]))[:80]
    return re.split(r"[(<]", n)[0][:80]
mq = max(byq.values(), key=len)
per = len(mq) // steps
print(f"\n--- main queue, last step ({per} kernels) ---")
prev = None
for r in mq[-per:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    print(f"{(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {short(r)}")

# other queues over the last two steps, start/end relative to the start of the main queue's
# second-to-last step (where crop formation overlaps the training step)
if len(byq) > 1:
    t0 = int(mq[-2 * per]["Start_Timestamp"])
    print(f"\n--- main step boundaries (us from t0) ---")
    for j in (2, 1):
        a, z = mq[-j * per], mq[-(j - 1) * per - 1]
        print(f"main step -{j}: {(int(a['Start_Timestamp']) - t0) / 1e3:8.1f} .. {(int(z['End_Timestamp']) - t0) / 1e3:8.1f}")
    for q, rs in byq.items():
        if rs is mq:
            continue
        print(f"--- queue {q}, kernels starting after t0 ---")
        for r in rs:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if s >= t0:
                print(f"{(s - t0) / 1e3:8.1f} .. {(e - t0) / 1e3:8.1f}  {(e - s) / 1e3:7.1f} us  {short(r)}")
    print("--- main queue: kernels starting after t0 with a gap > 10 us before them ---")
    prev = None
    for r in mq:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s >= t0 and prev is not None and s - prev > 10000:
            print(f"{(s - t0) / 1e3:8.1f}  gap {(s - prev) / 1e3:7.1f}  {short(r)}")
        prev = e
