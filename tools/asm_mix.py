"""Instruction mix per kernel of a hipcc -save-temps .s (dev tool)."""
import collections
import re
import sys

s = open(sys.argv[1]).read().split("\n")
starts = [(i, l.split(":")[0]) for i, l in enumerate(s) if re.match(r"^_ZN\w+:", l)]
starts.append((len(s), None))
for (a, name), (b, _) in zip(starts, starts[1:]):
    c = collections.Counter()
    for l in s[a:b]:
        if not l.startswith("\t") or l.strip().startswith((".", ";")):
            continue
        i = l.strip().split()[0]
        if i.startswith("v_mfma"): c["mfma"] += 1
        elif i.startswith("ds_"): c["ds"] += 1
        elif i.startswith(("global_load", "buffer_load", "flat_load")): c["vmem_ld"] += 1
        elif i.startswith(("global_store", "buffer_store", "flat_store")): c["vmem_st"] += 1
        elif "atomic" in i: c["atomic"] += 1
        elif i.startswith("s_waitcnt"): c["waitcnt"] += 1
        elif i.startswith(("s_cbranch", "s_branch")): c["branch"] += 1
        elif i.startswith("s_"): c["salu"] += 1
        elif i.startswith("v_"): c["valu"] += 1
        elif i.startswith("scratch"): c["scratch"] += 1
    print(f"{name[:44]:44s} {sum(c.values()):6d} {dict(c)}")
