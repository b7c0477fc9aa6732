"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (mean per dispatch)."""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/**/run_counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"]
        agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
out = {}
for k, cs in agg.items():
    short = k.split("(")[0].replace("void ", "").replace("tt::", "")
    out[short] = {c: sum(v) / len(v) for c, v in cs.items()}
    if len(sys.argv) > 2 and sys.argv[2] not in short:
        continue
for k in sorted(out):
    if "tt" not in k and "k_" not in k:
        continue
    print(k, json.dumps({c: round(v) for c, v in sorted(out[k].items())}))
