"""Per-epoch device timeline of a train_model run (rocprofv3 --kernel-trace
--memory-copy-trace csv): epochs delimited by the k_l0_fwd launches (611 per
cfg-3 epoch), wall vs kernel-busy time per epoch, and the host-to-device
copies of >= 1 ms with what ran beside them.
usage: python tools/epoch_windows.py <dir> [steps_per_epoch]"""
import bisect
import csv
import glob
import sys

d = sys.argv[1]
spe = int(sys.argv[2]) if len(sys.argv) > 2 else 611
ks, cp = [], []
for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
    ks += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in csv.DictReader(open(f))]
for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
    cp += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))]
ks.sort()
cp.sort()
t0 = ks[0][0]
l0 = [k for k in ks if "k_l0_fwd" in k[2]]
# the last call's epochs: the last 5 * spe l0 launches, in epoch-sized groups
for e in range(len(l0) // spe - 5, len(l0) // spe):
    a = l0[e * spe][0]
    b = l0[(e + 1) * spe][0] if (e + 1) * spe < len(l0) else ks[-1][1]
    busy = sum(min(k[1], b) - max(k[0], a) for k in ks if k[1] > a and k[0] < b)
    copies = [(s, t) for s, t in cp if a <= s < b and t - s > 1_000_000]
    print(f"epoch {e}: wall {1e-6 * (b - a):.3f} ms, kernels {1e-6 * busy:.3f} ms, "
          f"{1e-3 * (b - a) / spe:.2f} us/step; big H2D copies {[round((t - s) / 1e3) for s, t in copies]} us")
starts = [k[0] for k in ks]
for s, t in cp:
    if t - s < 1_000_000:
        continue
    i, j = bisect.bisect_left(starts, s), bisect.bisect_left(starts, t)
    print(f"copy @{1e-6 * (s - t0):.2f} ms, {1e-3 * (t - s):.0f} us, kernels beside it: {j - i}")
