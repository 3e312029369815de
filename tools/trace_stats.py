"""Per-kernel duration statistics from rocprofv3 --kernel-trace CSVs: launches, mean / median / p10 /
min duration and the median gap to the previous launch of the same kernel (back-to-back launches
under the tracer report gap 0: the recorded duration then spans the launch period).

    python tools/trace_stats.py <dir with *kernel_trace.csv> [name-substring ...]"""
import csv
import glob
import statistics as st
import sys


def stats(d, names=()):
    fs = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not fs:
        return {}
    by = {}
    for r in csv.DictReader(open(fs[0])):
        n = r["Kernel_Name"]
        if names and not any(x in n for x in names):
            continue
        by.setdefault(n.split("(")[0], []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for n, v in by.items():
        v.sort()
        durs = sorted((e - s) / 1000 for s, e in v)
        gaps = [(v[i + 1][0] - v[i][1]) / 1000 for i in range(len(v) - 1)]
        out[n] = dict(launches=len(durs), mean=st.mean(durs), median=st.median(durs), p10=durs[len(durs) // 10],
                      min=durs[0], gap_median=st.median(gaps) if gaps else 0.0)
    return out


if __name__ == "__main__":
    for n, s in stats(sys.argv[1], sys.argv[2:]).items():
        print(f"{n[-70:]:70s} " + " ".join(f"{k} {v:.3f}" if isinstance(v, float) else f"{k} {v}" for k, v in s.items()))
