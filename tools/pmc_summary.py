#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over the pmc_<tag>_* pass directories.

    python tools/pmc_summary.py <tag> [root] [--json out.json]

HBM bytes per launch follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so `hbm_read_bytes` doubles it
(an upper-bound correction for this workload's mix of widths); WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

argv = sys.argv[1:]
if "--json" in argv:  # the option's value is not a positional argument
    del argv[argv.index("--json") + 1]
args = [a for a in argv if not a.startswith("--")]
tag = args[0] if args else "r1"
root = args[1] if len(args) > 1 else "gpurun_out"
out_json = sys.argv[sys.argv.index("--json") + 1] if "--json" in sys.argv else None
acc = defaultdict(lambda: defaultdict(list))
grids = defaultdict(set)
for f in sorted(glob.glob(os.path.join(root, f"pmc_{tag}_*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        # drop namespaces before cutting at the argument list: argument types carry "::" too
        # (k_rnn_act(pm::ActGrid, ...)), and so do template arguments (k_env_step<2, false>)
        short = name.replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        short = short.split("::")[-1].strip()
        short = short[5:] if short.startswith("void ") else short
        grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "0"
        acc[f"{short}@{grid}"][r["Counter_Name"]].append(float(r["Counter_Value"]))
        grids[short].add(int(grid))
# a kernel launched with several grids (k_act_sp: full act / side B only; k_learn: with and without
# the side-A act blocks) is listed per grid as name@grid; the bare name is its LARGEST grid
for short, gs in grids.items():
    acc[short] = acc[f"{short}@{max(gs)}"]
keys = ["k_act_sp", "k_env", "k_learn", "k_env_step"]
summary = {}
for k in keys + sorted(set(acc) - set(keys)):
    if k not in acc:
        continue
    d = {c: sum(v) / len(v) for c, v in acc[k].items()}
    if "FETCH_SIZE" in d:
        d["hbm_read_bytes"] = d["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in d:
        d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
    if "hbm_read_bytes" in d and "hbm_write_bytes" in d:
        d["hbm_bytes"] = d["hbm_read_bytes"] + d["hbm_write_bytes"]
    summary[k] = d
    print(k, " ".join(f"{c}={d[c]:.4g}" for c in sorted(d)))
if out_json:
    with open(out_json, "w") as fh:
        json.dump({"tag": tag, "kernels": summary}, fh, indent=1, sort_keys=True)
