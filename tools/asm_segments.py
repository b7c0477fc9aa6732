"""Instruction mix of one kernel split at its s_memrealtime stamps (dev tool).
usage: python tools/asm_segments.py file.s kernel_substring"""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_ZN\w+:", l)] + [(len(s), None)]
for (a, n), (b, _) in zip(starts, starts[1:]):
    if sys.argv[2] not in n:
        continue
    print(n)
    segs, c = [], collections.Counter()
    for l in s[a:b]:
        if not l.startswith("\t") or l.strip().startswith((".", ";")):
            continue
        i = l.strip().split()[0]
        if i == "s_memrealtime":
            segs.append(c)
            c = collections.Counter()
            continue
        key = ("mfma" if i.startswith("v_mfma") else "bperm" if "bpermute" in i else "ds_add" if i.startswith("ds_add")
               else "ds" if i.startswith("ds_") else "vmem" if i.startswith(("global_", "buffer_"))
               else "wait" if i.startswith("s_waitcnt") else "br" if i.startswith("s_cbranch")
               else "salu" if i.startswith("s_") else "dpp" if "dpp" in l or "row_" in l else "valu" if i.startswith("v_") else "other")
        c[key] += 1
        if "_dpp" in i or "row_" in l or "quad_perm" in l:
            c["dpp"] += 1
    segs.append(c)
    for k, cc in enumerate(segs):
        print(f"  seg{k}: {sum(cc.values()):5d} {dict(cc)}")
    break
