"""Per-step kernel summary of bench.py's TIMED steps only (rocprofv3 --kernel-trace CSV): the
window runs from the end of the clip + RMSprop launch that precedes the first timed step to the
end of the last one, so the PipelinedTrainer's eager warm-up steps, the pose check and the
probe steps fall outside it. Kernels on both streams inside the window are counted (training
graphs on one, crop formation + deferred IR on the other); per step = window total / steps.

  python tools/step_window_summary.py kernel_trace.csv bench.json > summary.txt
"""
import collections
import csv
import json
import re
import sys


def short(n):
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"^void ", "", n)
    out, depth = "", 0
    for ch in n:
        if ch == "(" and depth == 0 and out:
            break
        out += ch
        depth += ch == "<"
        depth -= ch == ">"
    return out[:72]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    steps = int(bench["steps"])
    marks = [r for r in rows if "clip_rmsprop_kernel" in r["Kernel_Name"]]
    if len(marks) < steps + 1:
        sys.exit(f"only {len(marks)} clip_rmsprop launches for {steps} steps")
    lo, hi = int(marks[-steps - 1]["End_Timestamp"]), int(marks[-1]["End_Timestamp"])
    win = [r for r in rows if int(r["Start_Timestamp"]) >= lo and int(r["End_Timestamp"]) <= hi]
    queues = collections.Counter(r.get("Queue_Id", r.get("Stream_Id", "?")) for r in win)
    tot = collections.defaultdict(lambda: [0, 0])
    for r in win:
        t = tot[short(r["Kernel_Name"])]
        t[0] += 1
        t[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(v[1] for v in tot.values())
    print(f"timed window {steps} steps, {(hi - lo) / 1e6:.3f} ms ({(hi - lo) / 1e3 / steps:.1f} us per step; bench "
          f"{bench['ms_per_step'] * 1e3:.1f}); kernel time {busy / 1e3 / steps:.1f} us per step over "
          f"{len(queues)} queues ({', '.join(str(c // steps) for c in queues.values())} launches per step)")
    print(f"{'kernel':72s}{'/step':>6s} {'avg us':>8s} {'us/step':>9s}")
    for name, (n, ns) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{name:72s}{n / steps:6.1f} {ns / n / 1e3:8.2f} {ns / 1e3 / steps:9.1f}")
    # where torch's own kernels sit: queue and the launches before / after on the same queue
    byq = collections.defaultdict(list)
    for r in win:
        byq[r.get("Queue_Id", r.get("Stream_Id", "?"))].append(r)
    ctx = collections.Counter()
    for q, rs in byq.items():
        for i, r in enumerate(rs):
            if "at::" in r["Kernel_Name"] or "rocclr" in r["Kernel_Name"]:
                prev = short(rs[i - 1]["Kernel_Name"]) if i > 0 else "-"
                nxt = short(rs[i + 1]["Kernel_Name"]) if i + 1 < len(rs) else "-"
                ctx[(q, short(r["Kernel_Name"]), prev, nxt)] += 1
    # one step's launch sequence per queue (the last timed step: between the last two markers)
    lo2 = int(marks[-2]["End_Timestamp"])
    for q, rs in sorted(byq.items(), key=lambda kv: -len(kv[1])):
        seq = [r for r in rs if int(r["Start_Timestamp"]) >= lo2]
        print(f"\nqueue {q}: {len(seq)} launches in the last step")
        for r in seq:  # duration, then start / end relative to the step's start (the last clip_rmsprop end)
            print(f"  {(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3:8.2f}  {short(r['Kernel_Name']):60s}"
                  f" @ {(int(r['Start_Timestamp']) - lo2) / 1e3:8.1f} .. {(int(r['End_Timestamp']) - lo2) / 1e3:8.1f}")
    # head of every training replay: the first main-queue kernel after each clip + RMSprop, its
    # start against the previous step's end and against the crop-formation stream's last kernel
    # before it (the formed[k] event the replay waits on), and its duration
    mq = max(byq.items(), key=lambda kv: len(kv[1]))[0]
    side = [r for q, rs in byq.items() if q != mq for r in rs]
    print("\nhead of each training replay (us): start - previous clip_rmsprop end, start - last side-queue "
          "kernel end before it (negative: the head started before crop formation finished), duration")
    mains = byq[mq]
    for i, r in enumerate(mains):
        if i == 0 or "clip_rmsprop_kernel" not in mains[i - 1]["Kernel_Name"]:
            continue
        st, prev_end = int(r["Start_Timestamp"]), int(mains[i - 1]["End_Timestamp"])
        before = [int(x["End_Timestamp"]) for x in side if int(x["Start_Timestamp"]) < st]
        last_side = max(before) if before else None
        dur = int(r["End_Timestamp"]) - st
        sk = [x for x in side if int(x["End_Timestamp"]) == last_side]
        print(f"  {short(r['Kernel_Name'])[:40]:40s} gap {(st - prev_end) / 1e3:8.2f}  vs side "
              f"{(st - last_side) / 1e3 if last_side else float('nan'):8.2f} ({short(sk[0]['Kernel_Name'])[:24] if sk else '-'})"
              f"  dur {dur / 1e3:8.2f}")
    if ctx:
        print("\ntorch / runtime kernels in the window (queue, kernel, previous, next):")
        for (q, k, a, b), c in sorted(ctx.items(), key=lambda kv: -kv[1]):
            print(f"  q{q} x{c / steps:.1f}/step  {k[:50]}  after {a[:40]}  before {b[:40]}")


if __name__ == "__main__":
    main()
