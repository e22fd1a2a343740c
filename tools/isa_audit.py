"""ISA audit of every kernel of libposekern (hipcc -S output directory): per kernel the global
loads, the loads directly behind an exec-mask branch (a conditional load: the compiler waits for
it before the branch rejoins, serialising memory round trips), and vmcnt(0) waits.
python tools/isa_audit.py <dir of .s files> [top]"""
import glob
import re
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/*.s"):
    s = open(f).read()
    for m in re.finditer(r"^(_Z\w+):", s, re.M):
        name = m.group(1)
        end = s.find(".Lfunc_end", m.end())
        body = s[m.end():end]
        lines = body.splitlines()
        gl = sum(1 for l in lines if l.strip().startswith("global_load"))
        w0 = sum(1 for l in lines if "vmcnt(0)" in l)
        guarded = 0
        for i, l in enumerate(lines):
            if "s_cbranch_execz" in l and any(x.strip().startswith("global_load") for x in lines[i + 1:i + 4]):
                guarded += 1
        if gl:
            rows.append((guarded, gl, w0, f.split("/")[-1], re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)[:70]))
rows.sort(reverse=True)
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print("guarded_loads global_loads vmcnt0_waits file kernel")
for r in rows[:top]:
    print(*r)
