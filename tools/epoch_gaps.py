"""Gaps in the device timeline of a train_model run (rocprofv3 --kernel-trace
--memory-copy-trace csv): per gap > 2 us between consecutive device
operations, what ended before and what started after; totals per kind.
usage: python tools/epoch_gaps.py <dir with run_kernel_trace.csv>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
ev = []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "?")))
ev.sort()
# steady region: from the 2nd occurrence of a long run of k_l0_fwd after the first copy of >1 ms
t0, t1 = ev[0][0], ev[-1][1]
gaps = collections.Counter()
gapn = collections.Counter()
busy = collections.Counter()
end = ev[0][1]
prev = ev[0][2]
big = []
for s, e, n in ev[1:]:
    busy[n] += e - s
    if s - end > 2000:
        gaps[(prev, n)] += s - end
        gapn[(prev, n)] += 1
        big.append((s - end, prev, n))
    if e > end:
        end, prev = e, n
print(f"span {1e-6 * (t1 - t0):.2f} ms, ops {len(ev)}")
print("device time by op (ms):", {k: round(v * 1e-6, 3) for k, v in busy.most_common(12)})
print("gaps > 2 us by (before, after): total ms, count")
for k, v in gaps.most_common(12):
    print(f"  {k}: {v * 1e-6:.3f} ms, {gapn[k]}")
print("largest gaps (us):", [(round(g / 1e3, 1), a, b) for g, a, b in sorted(big, reverse=True)[:10]])
