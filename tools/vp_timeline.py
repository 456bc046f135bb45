"""VerifyProposal (config 3) GPU timeline from a rocprofv3 kernel + memory-copy trace of
tools/latency_probe.py-style calls: per call, the copies and kernels with their start offsets
and durations relative to the call's first copy (diagnostics for DESIGN.md)."""
import csv
import glob
import sys


def load(d):
    ev = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:]))
    for f in glob.glob(f"{d}/**/*memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?") + " " + r.get("Size", "")))
    return sorted(ev)


ev = load(sys.argv[1])
# calls: the pair kernel marks each VerifyProposal; show the events around the last few
idx = [i for i, e in enumerate(ev) if "small_kernel" in e[2]]
for k in idx[-3:]:
    lo = k
    while lo > 0 and ev[k][0] - ev[lo - 1][0] < 400_000:  # 0.4 ms before the verify kernel
        lo -= 1
    hi = k
    while hi + 1 < len(ev) and ev[hi + 1][0] - ev[k][1] < 100_000:
        hi += 1
    t0 = ev[lo][0]
    print("---")
    for s, e, name in ev[lo:hi + 1]:
        print(f"{(s - t0) / 1e3:9.1f} us  +{(e - s) / 1e3:8.1f} us  {name}")
