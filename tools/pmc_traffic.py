"""HBM traffic per kernel launch from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

    python tools/pmc_traffic.py gpurun_out/<tag> [profiles/pmc_traffic.json]

Reads the FETCH_SIZE and WRITE_SIZE passes written by tools/pmc_profile.sh
(separate --pmc runs: the two TCC counters do not fit one pass on gfx950) and
applies the MI355X guide's corrections (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the
bytes of wide (16 B/lane) coalesced reads -- every hot read of this path is a
16-B-per-lane load -- so fetched bytes = 2 * 1024 * FETCH_SIZE; WRITE_SIZE is
exact for 16-B stores and float atomics.  Values are means over dispatches,
per kernel name ("kernels", what bench.py reads) and per template instance
("instances").  tools/pmc_profile.sh runs the headline config only, so a
kernel name does not mix two configs' launches.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").strip()
    n = re.sub(r"<.*>", "", n)
    return n.split("::")[-1]


def instance(name):
    n = name.split("(")[0].replace("void ", "").strip()
    head, _, targs = n.partition("<")
    return head.split("::")[-1] + ("<" + targs if targs else "")


def collect(root, key=short):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            agg[key(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return agg


def traffic(agg):
    kernels = {}
    for k, cs in sorted(agg.items()):
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
        w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
        kernels[k] = {
            "dispatches": len(cs["FETCH_SIZE"]),
            "FETCH_SIZE_kib": round(f, 1),
            "WRITE_SIZE_kib": round(w, 1),
            "read_bytes_per_launch": round(2 * 1024 * f),
            "write_bytes_per_launch": round(1024 * w),
            "hbm_bytes_per_launch": round(2 * 1024 * f + 1024 * w),
        }
    return kernels


def main():
    root = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                   "pmc_traffic.json")
    kernels = traffic(collect(root))
    # the build the counters describe: bench.py marks roofline.traffic stale
    # when the library it loaded is another one
    import hashlib
    lib = os.environ.get("CEO_TT_LIB") or os.path.join(os.path.dirname(__file__), "..", "ceo-recommender_amd",
                                                       "lib", "libceo_tt.so")
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest() if os.path.exists(lib) else None
    doc = {
        "source": os.path.basename(os.path.normpath(root)),
        "library_sha256": sha,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes); "
                  "bytes = 2*1024*FETCH_SIZE + 1024*WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md HBM)",
        "kernels": kernels,
        "instances": traffic(collect(root, instance)),
    }
    with open(out_path, "w") as fh:
        json.dump(doc, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k:16s} {v['hbm_bytes_per_launch'] / 1e6:9.2f} MB/launch  (n={v['dispatches']})")


if __name__ == "__main__":
    main()
