"""Per-kernel statistics (calls, total / average / min / max ns, share) from a rocprofv3 SQLite
database (`rocprofv3 --kernel-trace ... -o run` writes run_results.db), as CSV on stdout.

    python tools/rocpd_stats.py gpurun_out/prof_rnn/run_results.db [--grid]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--grid", action="store_true", help="split kernels by grid size")
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    names = {i: (dn or kn) for i, kn, dn in cur.execute(f"select id, kernel_name, display_name from {ks}")}
    acc = collections.defaultdict(list)
    for kid, s, e, gx in cur.execute(f"select kernel_id, start, end, grid_size_x from {kd}"):
        key = names.get(kid, str(kid))
        if a.grid:
            key = f"{key} [grid {gx}]"
        acc[key].append(e - s)
    total = sum(sum(v) for v in acc.values())
    print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage")
    for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f'"{k}",{len(v)},{sum(v)},{sum(v) / len(v):.1f},{min(v)},{max(v)},{100.0 * sum(v) / total:.2f}')


if __name__ == "__main__":
    main()
