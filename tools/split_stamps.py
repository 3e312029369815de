"""Timeline of configs[4]'s side-A act launch (diagnostic library): after one overlapped RNN
self-play step at 32 768 arenas (pool 4, the bench's workload), the whole-group blocks' start / end
(rnn_group's ring stamps, slot 0 and 46) and the split tiles' phases (rnn_tile_split, slots 48..61),
in us from the launch's first block start.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/split_stamps.py
"""
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

SPLIT = ["start", "F2 done", "F2 exchanged", "gates m0", "cell m0", "gates m1", "cell m1", "gates m2", "cell m2",
         "gates m3", "cell m3", "heads stage done", "S exchanged", "end"]


def main():
    import bench
    from pongmi import _lib
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    lib = _lib.load()
    lib.pm_diag_read_rnn.argtypes = [ctypes.c_void_p]
    L = RNNSelfPlayLearner(bench.ENV_KW_RNN, 32768, bench.synthetic_rnn(1), bench.synthetic_rnn(2),
                           [bench.synthetic_rnn(100 + k) for k in range(4)], epsilon=0.05, seed=7)
    for _ in range(70):
        L.step()
    torch.cuda.synchronize()
    rows = []
    for rep in range(3):
        lib.pm_diag_clear_rnn()
        L.step()
        torch.cuda.synchronize()
        buf = (ctypes.c_uint64 * (64 * 1024))()
        lib.pm_diag_read_rnn(buf)
        st = np.array(buf[:], dtype=np.int64).reshape(64, 1024)
        whole = np.nonzero((st[0] > 0) & (st[46] > 0) & (st[48] == 0))[0]
        split = np.nonzero(st[48] > 0)[0]
        t0 = min(st[0][whole].min() if len(whole) else 1 << 62, st[48][split].min() if len(split) else 1 << 62)
        us = lambda a: (a - t0) / 100.0  # noqa: E731  100 MHz
        print(f"step {rep}: {len(whole)} whole-group blocks, {len(split)} split-tile blocks")
        if len(whole):
            print(f"  whole groups: start p50 {np.median(us(st[0][whole])):.1f}  end p50 {np.median(us(st[46][whole])):.1f}"
                  f"  end max {us(st[46][whole]).max():.1f} us")
        if len(split):
            s = st[48:48 + len(SPLIT)][:, split]
            print(f"  split tiles: start min {us(s[0]).min():.1f} p50 {np.median(us(s[0])):.1f} max {us(s[0]).max():.1f};"
                  f" end p50 {np.median(us(s[-1])):.1f} max {us(s[-1]).max():.1f} us")
            d = np.diff(s, axis=0) / 100.0
            for k in range(1, len(SPLIT)):
                print(f"    {SPLIT[k - 1]:>16s} -> {SPLIT[k]:<16s} p50 {np.median(d[k - 1]):6.2f}  max {d[k - 1].max():6.2f} us")
            rows.append(np.median((s[-1] - s[0]) / 100.0))
    if rows:
        print(f"split tile duration p50 over steps: {np.median(rows):.1f} us")


if __name__ == "__main__":
    main()
