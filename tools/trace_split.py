#!/usr/bin/env python3
"""Per-kernel, per-grid launch durations from a rocprofv3 --kernel-trace CSV (k_kernel_trace.csv):
one kernel launched with two geometries (k_rnn_act: modelB's side on the full grid, the opponents'
side on the capped grid beside the DRQN update) splits into one line per geometry.

    python3 tools/trace_split.py gpurun_out/prof_rnn_r2d/k_kernel_trace.csv [name-substring ...]
"""
import collections
import csv
import sys


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if keys and not any(k in name for k in keys):
            continue
        grid = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Workgroup_Size_X"]))
        short = name.replace("(anonymous namespace)::", "").split("(")[0]
        groups[(short, grid)].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    print(f"{'kernel':60s} {'blocks':>7s} {'threads':>7s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s}")
    for (name, (blocks, threads)), v in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:60]:60s} {blocks:7d} {threads:7d} {len(v):6d} {sum(v) / len(v):9.2f} {min(v):9.2f} {max(v):9.2f}")


if __name__ == "__main__":
    main()
