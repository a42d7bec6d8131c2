"""Static instruction mix of the fr_expand instantiations in a hipcc -S dump (tool).
usage: hipcc --offload-arch=gfx950 -O3 -std=c++17 --cuda-device-only -S csrc/frontier.hip -o /tmp/fr.s; isa_mix.py /tmp/fr.s [substr]"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split("\n")
want = sys.argv[2] if len(sys.argv) > 2 else "fr_expand"
i = 0
while i < len(L):
    m = re.match(r"^(_Z\w+):", L[i])
    if m and want in m.group(1):
        name = m.group(1)
        ins = []
        i += 1
        while i < len(L) and not L[i].startswith(".Lfunc_end"):
            t = L[i].strip()
            if L[i].startswith("\t") and t and not t.startswith((".", ";")):
                ins.append(t.split()[0])
            i += 1
        c = collections.Counter(ins)
        cat = collections.Counter()
        for op, n in c.items():
            if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
                cat["v_lane"] += n
            elif op.startswith("v_"):
                cat["valu"] += n
            elif op.startswith("s_"):
                cat["salu"] += n
            elif op.startswith("ds_"):
                cat["lds"] += n
            elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
                cat["vmem"] += n
        print(f"{name[:70]:70s} {len(ins):6d} " + " ".join(f"{k}={v}" for k, v in sorted(cat.items())))
    i += 1
