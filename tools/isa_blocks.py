"""Basic blocks of one kernel in a hipcc -S output: label, instruction counts (MFMA, VALU, SALU,
DS, VMEM, s_nop), and the branch that ends the block; with --dump LABEL the block's pattern
(M = MFMA, v = VALU, s = SALU, d = DS, g = global).
  python tools/isa_blocks.py file.s kernel_substring [--dump .LBBx_y]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
m = re.search(r"^(_Z\w*%s\w*):" % sys.argv[2], s, re.M)
end = s.find(".Lfunc_end", m.end())
lines = [l.strip() for l in s[m.end():end].splitlines() if l.strip() and not l.strip().startswith(";")]
blocks, cur, name = [], [], "entry"
for l in lines:
    if re.match(r"^\.LBB\d+_\d+:", l):
        blocks.append((name, cur))
        name, cur = l[:-1], []
    elif not l.startswith("."):
        cur.append(l)
blocks.append((name, cur))
dump = sys.argv[sys.argv.index("--dump") + 1] if "--dump" in sys.argv else None
for name, b in blocks:
    c = Counter("M" if t.startswith("v_mfma") else "n" if t.startswith("s_nop") else t[0] if t[0] in "vsdg" else "?" for t in b)
    br = [t for t in b if t.startswith("s_branch") or t.startswith("s_cbranch")]
    print(f"{name:10s} n={len(b):4d} mfma={c['M']:3d} valu={c['v']:4d} salu={c['s']:4d} nop={c['n']:3d} ds={c['d']:3d} "
          f"gl={c['g']:3d}  {br[-1] if br else ''}")
    if name == dump:
        print("".join("M" if t.startswith("v_mfma") else "n" if t.startswith("s_nop") else t[0] for t in b))
        if "--full" in sys.argv:
            print("\n".join(b))
