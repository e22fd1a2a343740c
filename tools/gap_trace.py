"""Gaps on the training stream of bench.py's overlapped step (rocprofv3 kernel trace): each idle
interval longer than a threshold, the kernels before / after it and the side-stream kernel(s)
running meanwhile. python tools/gap_trace.py trace.csv bench.log [min_gap_us]"""
import collections, csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
bench = next(json.loads(l) for l in reversed(open(sys.argv[2]).read().splitlines()) if l.startswith('{"metric"'))
steps = int(bench["steps"])
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0
t1 = max(int(r["End_Timestamp"]) for r in rows)
lo = t1 - int(steps * bench["ms_per_step"] * 1e6)
win = [r for r in rows if int(r["Start_Timestamp"]) >= lo]
byq = collections.defaultdict(list)
for r in win:
    byq[r.get("Queue_Id", r.get("Stream_Id", "?"))].append(r)
qs = sorted(byq, key=lambda q: -len(byq[q]))
main, side = qs[0], qs[1] if len(qs) > 1 else None
short = lambda n: n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]  # noqa: E731
agg = collections.Counter()
tot = collections.Counter()
prev = None
for r in byq[main]:
    s = int(r["Start_Timestamp"])
    if prev is not None and (s - int(prev["End_Timestamp"])) / 1e3 > thr:
        g0, g1 = int(prev["End_Timestamp"]), s
        during = [short(x["Kernel_Name"]) for x in byq[side] if int(x["Start_Timestamp"]) < g1 and int(x["End_Timestamp"]) > g0] if side else []
        key = (short(prev["Kernel_Name"]), short(r["Kernel_Name"]), ",".join(sorted(set(during))))
        agg[key] += 1
        tot[key] += (g1 - g0) / 1e3
    prev = r
print(f"main queue {main}, side {side}, {steps} steps; gaps > {thr} us:")
for k, n in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{n / steps:8.1f} us/step  x{agg[k] / steps:.1f}  after {k[0]:40s} before {k[1]:40s} side: {k[2]}")

# one step's timeline (the middle step of the window): both queues, start offset / duration in us
mid = lo + (steps // 2) * int(bench["ms_per_step"] * 1e6)
t0 = mid
t1s = mid + int(bench["ms_per_step"] * 1e6)
print("\ntimeline of one step (us from its start): queue, start, duration, kernel")
ev = [r for r in win if t0 <= int(r["Start_Timestamp"]) < t1s]
for r in ev:
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    s0 = (int(r["Start_Timestamp"]) - t0) / 1e3
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{'M' if q == main else 'S'} {s0:8.1f} {d:7.1f}  {short(r['Kernel_Name'])}")
