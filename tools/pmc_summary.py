#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel over the pmc_<tag>_* pass directories."""
import csv
import glob
import os
import sys
from collections import defaultdict

tag = sys.argv[1] if len(sys.argv) > 1 else "r1"
root = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, f"pmc_{tag}_*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.split("::")[-1].split("(")[0] if "::" in name else name.split("(")[0]
        acc[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
keys = ["k_act_sp", "k_env", "k_per_refresh", "k_sp_sample", "k_dqn_fwd", "k_dqn", "k_env_step"]
for k in keys + sorted(set(acc) - set(keys)):
    if k not in acc:
        continue
    d = {c: sum(v) / len(v) for c, v in acc[k].items()}
    print(k, " ".join(f"{c}={d[c]:.4g}" for c in sorted(d)))
