"""Phase timeline of k_learn_multi (diagnostic library): thread 0's s_memrealtime stamps of the last
update of a vector step, relative to that update's start.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/multi_stamps.py [--U 16]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.environ.get("PONGMI_DIAG_LIB") or os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi",
                                                                             "libpongmi_diag.so")
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = {111: "  level-2 search done", 112: "  level 1 (16 sub sums)", 113: "  level 0 (64 leaves)",
         115: "  grads + Adam done", 117: "  rows landed", 118: "  chains done", 116: "  level-1 leaves loaded",
         101: "prefix", 102: "heads (row gather + chains)", 103: "IS weights (pow) + wmax", 104: "wmax",
         105: "TD / hash", 106: "scatter + grad partials", 107: "grads + Adam + level-1 refresh",
         108: "level 2 + target sync", 109: "derive weights", 100: "next update start",
         119: "  hash table cleared", 120: "  chunk sums (4 per lane)", 121: "  fp64 wave scan", 122: "  first barrier",
         124: "update end (last barrier)"}


ORDER = [119, 120, 121, 122, 101, 111, 112, 113, 117, 118, 102, 103, 104, 105, 106, 115, 116, 107, 108, 109, 124]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--U", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    args = ap.parse_args()
    import bench
    from pongmi import _lib
    from pongmi.selfplay import SelfPlayLearner
    lib = _lib.load()
    lib.pm_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    L = SelfPlayLearner(bench.ENV_KW, 65536, sdB, sdA, pool, batch=256, memory_size=1_000_000, epsilon=0.08, seed=7,
                        updates_per_step=args.U)
    for _ in range(10):
        L.step()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 256)()
    rows = []
    for _ in range(args.steps):
        lib.pm_diag_clear()
        L.step()
        torch.cuda.synchronize()
        lib.pm_diag_read(buf, 256)
        v = np.array(buf[:256], dtype=np.int64)
        rows.append([(v[k] - v[100]) / 100.0 for k in ORDER])  # 100 MHz -> us
    med = np.median(np.array(rows), 0)
    prev = 0.0
    for k, m in zip(ORDER, med):
        print(f"{NAMES[k]:34s} {m:8.2f} us  (+{m - prev:6.2f})")
        prev = m


if __name__ == "__main__":
    main()
