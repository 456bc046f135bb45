"""Per-dispatch summary of a rocprofv3 --kernel-trace CSV (run_kernel_trace.csv) for one kernel:
every dispatch of the bench's full-size grid in order, the mean over all of them (what the
--stats table averages), and the mean over the last STEPS dispatches -- the timed steps that
bench.py's HIP events cover -- so that the profile and the bench line can be compared on the
same dispatches (the first full-size dispatch after start-up runs ~15% slow).

usage: python tools/trace_summary.py run_kernel_trace.csv KERNEL_SUBSTRING STEPS [GRID_X]
"""
import csv
import json
import sys


def main():
    path, name, steps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    grid = int(sys.argv[4]) if len(sys.argv) > 4 else None
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            if name not in r["Kernel_Name"]:
                continue
            if grid is not None and int(r["Grid_Size_X"]) != grid:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"]), r["Kernel_Name"]))
    rows.sort()
    if not rows:
        sys.exit(f"no dispatch of {name!r} in {path}")
    # the full-size dispatches are the ones with the largest grid
    big = max(g for _, _, g, _ in rows)
    full = [(e - s) / 1e6 for s, e, g, _ in rows if g == big]
    small = [(e - s) / 1e6 for s, e, g, _ in rows if g != big]
    timed = full[-steps:] if steps <= len(full) else full
    out = {
        "kernel": rows[0][3].split("(")[0],
        "grid_x": big,
        "full_size_dispatches": len(full),
        "dispatch_ms": [round(x, 4) for x in full],
        "mean_all_full_size_ms": round(sum(full) / len(full), 4),
        "mean_last_steps_ms": round(sum(timed) / len(timed), 4),
        "steps": len(timed),
        "other_grid_dispatches": len(small),
        "other_grid_mean_ms": round(sum(small) / len(small), 4) if small else None,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
