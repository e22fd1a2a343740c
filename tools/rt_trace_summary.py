"""Merge rocprofv3 kernel and HIP API traces: for the last few steps, graph launches and
event waits on the host timeline next to the first kernel each queue runs after them."""
import csv, glob, os, sys, re
d = sys.argv[1]
kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
af = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
ks = list(csv.DictReader(open(kf[0])))
api = list(csv.DictReader(open(af[0]))) if af else []
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
print("api columns:", list(api[0].keys()) if api else None)
names = {}
for a in api:
    names[a["Function"]] = names.get(a["Function"], 0) + 1
print("api counts:", sorted(names.items(), key=lambda kv: -kv[1])[:25])
interesting = [a for a in api if a["Function"] in ("hipGraphLaunch", "hipStreamWaitEvent", "hipEventRecord",
                                                    "hipEventRecordWithFlags", "hipStreamSynchronize",
                                                    "hipDeviceSynchronize", "hipEventSynchronize")]
t_end = int(ks[-1]["End_Timestamp"])
t0 = t_end - 4 * 3_000_000  # last ~4 steps
ev = [(int(a["Start_Timestamp"]), int(a["End_Timestamp"]), "API", a["Function"]) for a in interesting
      if int(a["Start_Timestamp"]) >= t0]
for r in ks:
    s = int(r["Start_Timestamp"])
    if s >= t0:
        n = re.split(r"[(<]", r["Kernel_Name"].replace("void ", ""))[0][-40:]
        ev.append((s, int(r["End_Timestamp"]), "Q" + r.get("Queue_Id", "?"), n))
ev.sort()
prev_q = {}
for s, e, kind, n in ev:
    if kind == "API":
        print(f"{(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f}  host  {n}")
    else:
        # print only the first kernel of a queue after a gap > 20 us, and big kernels
        g = s - prev_q.get(kind, s)
        if g > 20000 or e - s > 100000:
            print(f"{(s - t0) / 1e3:9.1f} .. {(e - t0) / 1e3:9.1f}  {kind:5s} {n}  (gap {g / 1e3:.1f})")
        prev_q[kind] = e
