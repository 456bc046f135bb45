"""Medians of the SBFT_VP_TRACE lines a split VerifyProposal run wrote to stderr (the engine's
`vp-split` share pick-up / end times and the call's `vp` phase line), microseconds from the call's
start. Usage: python tools/split_trace_summary.py TRACE_FILE"""
import re
import statistics
import sys


def main(path):
    split, calls = [], []
    for line in open(path):
        if line.startswith("vp-split"):
            d = {"start": float(re.search(r"start=([\d.]+)", line).group(1))}
            for i, a, b in re.findall(r"s(\d+)=([\d.-]+),([\d.-]+)", line):
                d[f"s{i}_pick"], d[f"s{i}_end"] = float(a), float(b)
            split.append(d)
        elif line.startswith("vp async"):
            calls.append({k: float(v) for k, v in re.findall(r"(\w+)=([\d.-]+)", line) if k != "async"})
    out = {}
    for name, rows in (("split", split), ("one_slot_calls", calls)):
        if rows:
            keys = rows[-1].keys()
            out[name] = {k: round(statistics.median(r[k] for r in rows if k in r), 1) for k in keys}
            out[name]["n"] = len(rows)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1])
