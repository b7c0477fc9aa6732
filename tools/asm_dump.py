"""Dump one s_memrealtime-delimited segment of a kernel's ISA (dev tool).
usage: python tools/asm_dump.py file.s kernel_substring seg"""
import re
import sys

s = open(sys.argv[1]).read().split("\n")
st = [i for i, l in enumerate(s) if re.match(r"^_ZN\w+:", l) and sys.argv[2] in l][0]
seg, want = 0, int(sys.argv[3])
for l in s[st + 1:]:
    if re.match(r"^_ZN\w+:", l) or l.strip().startswith("s_endpgm"):
        break
    if "s_memrealtime" in l:
        seg += 1
        continue
    if seg == want and (l.startswith("\t") and not l.strip().startswith((".", ";")) or l.startswith(".LBB")):
        print(l.strip())
