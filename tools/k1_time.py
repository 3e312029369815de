"""K1 (pm_env_step, autoreset 'done') launch time at several arena counts: graph-replayed
back-to-back launches, HIP events (bench.time_env_step). One JSON line per (n, repeat).

    python tools/k1_time.py [n ...]          (PONGMI_LIB=... selects an experimental build)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

for n in [int(a) for a in sys.argv[1:]] or [65536, 262144]:
    for rep in range(2):
        r = bench.time_env_step(n)
        print(json.dumps({"n": n, "rep": rep, "avg_us": r["avg_us"], "frac": r["frac"], "dispatch_us": r["dispatch_us"],
                          "dispatch_frac": r["dispatch_frac"]}), flush=True)
