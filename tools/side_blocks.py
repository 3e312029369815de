"""Timeline of k_learn's side blocks (configs[2], overlapped step, diagnostic library): the side-A act
blocks (the opponents' act for the next vector step) and the feature blocks (modelB's features of the
next observations), per role: begin, the act blocks' post-sleep start and end, relative to the learner
block's start (stamp 0), with the rows each block handled.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/side_blocks.py

Diagnostic only (libpongmi_diag.so, never the product library).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi", "libpongmi_diag.so")
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import bench
    from pongmi import _lib
    from pongmi.selfplay import SelfPlayLearner
    lib = _lib.load()
    lib.pm_diag_read_side.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    lib.pm_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    lib.pm_diag_read_blk.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    n = 65536
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    L = SelfPlayLearner(bench.ENV_KW, n, sdB, sdA, pool, batch=256, memory_size=1_000_000, epsilon=0.08, seed=7)
    for _ in range(40):
        L.step()
    torch.cuda.synchronize()
    # the host's learn_grid (pm_selfplay.hip), PONGMI_SIDE 1 (default) / 0, on a 256-CU device
    ntiles = (n + 31) // 32
    if os.environ.get("PONGMI_SIDE") == "0":
        c0, c1, ft = min(4 * L.sp.chunk_A, 4096), min(4 * L.sp.chunk_P, 4096), 16
    else:
        def chunk(p):
            return 16384 if p <= 0 else min(16384, max(256, -(-480 / p // 256) * 256))
        c0, c1 = int(chunk(1 - L.sp.pool_ratio)), int(chunk(L.sp.pool_ratio / 8))
    na0, na1 = (n + c0 - 1) // c0, (n + c1 - 1) // c1
    nact = na0 + 8 * na1
    if os.environ.get("PONGMI_SIDE") != "0":
        left = 256 - 2 - nact
        ft = min(max(-(-ntiles // left), 16), ntiles)
    nfeat = (ntiles + ft - 1) // ft
    side = (ctypes.c_uint64 * (4 * 1024))()
    buf = (ctypes.c_uint64 * 256)()
    rows, tiles = [], []
    blk = (ctypes.c_uint64 * (8 * 4096))()
    for _ in range(20):
        L.step()
        torch.cuda.synchronize()
        lib.pm_diag_read_side(side)
        lib.pm_diag_read(buf, 256)
        lib.pm_diag_read_blk(blk)  # act_block's PM_BLK stamps of the side-A blocks (grid blocks 2 ..)
        b = np.array(blk[:], dtype=np.int64).reshape(8, 4096)[:, 2:2 + nact]
        a = np.array(side[:], dtype=np.int64).reshape(4, 1024)[:, :nact + nfeat]
        t0 = int(buf[0])  # learner start
        rows.append(((a[0] - t0) * 0.01, (a[1] - t0) * 0.01, (a[2] - t0) * 0.01, a[3] >> 16))
        tiles.append(((b[4] - t0) * 0.01, (b[1] - t0) * 0.01, (b[5] - t0) * 0.01, (b[6] - t0) * 0.01,
                      (b[7] - t0) * 0.01))
    beg = np.median(np.stack([r[0] for r in rows]), axis=0)
    slp = np.median(np.stack([r[1] for r in rows]), axis=0)
    end = np.median(np.stack([r[2] for r in rows]), axis=0)
    cnt = rows[-1][3]
    print(f"k_learn side blocks: {na0} modelA act (chunk {c0}), {8 * na1} pool act (chunk {c1}), {nfeat} feature; "
          f"us from the learner block's start, median over 20 steps (min p50 p90 max)")

    def line(name, sel):
        for lab, v in (("begin", beg[sel]), ("start", slp[sel]), ("end", end[sel])):
            if lab == "start" and name == "feature":
                continue
            print(f"  {name:8s} {lab:5s} {v.min():7.2f} {np.median(v):7.2f} {np.percentile(v, 90):7.2f} {v.max():7.2f}")
        c = cnt[sel]
        print(f"  {name:8s} rows  {c.min():7d} {int(np.median(c)):7d} {int(np.percentile(c, 90)):7d} {c.max():7d}")
    idx = np.arange(nact + nfeat)
    line("modelA", idx < na0)
    line("pool", (idx >= na0) & (idx < nact))
    line("feature", idx >= nact)
    # act blocks' inner phases (block thread 0 = wave 0): staging issued, lists / compaction done +
    # barrier, wave 0's first tile operands landed, its hidden layers, its heads
    tl = [np.median(np.stack([r[k] for r in tiles]), axis=0) for k in range(5)]
    for name, sel in (("modelA", np.arange(nact) < na0), ("pool", np.arange(nact) >= na0)):
        for lab, v in zip(("staged", "listed", "tile0 in", "tile0 hid", "tile0 heads"), tl):
            x = v[sel]
            print(f"  {name:8s} {lab:11s} {x.min():7.2f} {np.median(x):7.2f} {np.percentile(x, 90):7.2f} {x.max():7.2f}")
    late = np.argsort(end)[-8:]
    print("  latest 8 blocks (side index, role, begin, end, rows):",
          [(int(i), "A" if i < na0 else ("P" if i < nact else "F"), round(float(beg[i]), 2), round(float(end[i]), 2),
            int(cnt[i])) for i in late])


if __name__ == "__main__":
    main()
