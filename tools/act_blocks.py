"""Per-block timeline of k_act_sp from the diagnostic library (PM_BLK stamps).

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/act_blocks.py [--overlap]

For each block role (PER sampler, side B, side A net 0, side A pool nets) prints quantiles of the
begin / ready (weights staged + rows compacted) / end times relative to the first block's begin,
plus the busiest CU's block count. Diagnostic only.
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
    n = 65536
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    overlap = "--overlap" in sys.argv  # the production step: k_act_sp runs the sampler + side B only
    L = SelfPlayLearner(bench.ENV_KW, n, sdB, sdA, pool, batch=256, memory_size=1_000_000, epsilon=0.08, seed=7,
                        overlap=overlap)
    for _ in range(40):
        L.step()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * (8 * 4096))()
    runs = []
    for _ in range(5):
        lib.pm_diag_clear()
        L.step()
        torch.cuda.synchronize()
        lib.pm_diag_read_blk(buf)
        runs.append(np.array(buf[:], dtype=np.int64).reshape(8, 4096))
    sp = L.sp
    nsb = (sp.batch + 63) // 64  # PER_BS samples per sampler block
    nb = (n + 255) // 256  # kChunkB
    na0 = (n + sp.chunk_A - 1) // sp.chunk_A
    na1 = (n + sp.chunk_P - 1) // sp.chunk_P
    total = nsb + nb + (0 if overlap else na0 + sp.n_pool * na1)
    print(f"blocks: sampler {nsb}, B {nb}, A0 {na0} (chunk {sp.chunk_A}), pool {sp.n_pool}x{na1} "
          f"(chunk {sp.chunk_P}); total {total}")
    roles = {"sampler": slice(0, nsb), "B": slice(nsb, nsb + nb)}
    if not overlap:
        roles.update({"A0": slice(nsb + nb, nsb + nb + na0), "pool": slice(nsb + nb + na0, total)})
    for r, a in enumerate(runs):
        t0 = a[0, :total].min()
        rel = (a[:3, :total] - t0) * 0.01
        print(f"run {r}: kernel span {rel[2].max():.2f} us")
        for name, sl in roles.items():
            b, rd, e = rel[0, sl], rel[1, sl], rel[2, sl]
            q = lambda v: " ".join(f"{x:6.2f}" for x in np.percentile(v, [0, 50, 90, 100]))  # noqa: E731
            st = (a[4, sl] - t0) * 0.01
            extra = (f" | staged-begin {q(st - b)} | ready-staged {q(rd - st)} | end-ready {q(e - rd)}"
                     if name != "sampler" else "")
            print(f"  {name:7s} begin {q(b)} | end {q(e)}{extra}")
            if name == "sampler":
                x4, x5, x6, x7 = ((a[k, sl] - t0) * 0.01 for k in (4, 5, 6, 7))
                print(f"          level2 {q(x4 - b)} | level1 {q(x5 - x4)} | leaves {q(x6 - x5)} | pow {q(x7 - x6)} | "
                      f"write-out {q(e - x7)}")
            if name != "sampler":
                x5, x6, x7 = ((a[k, sl] - t0) * 0.01 for k in (5, 6, 7))
                print(f"          tile0: obs-ready {q(x5 - rd)} | hidden {q(x6 - x5)} | heads {q(x7 - x6)}")
        place = a[3, :total]
        cu = place & 0xFFFF
        xcc = place >> 16
        ids = xcc * 1000 + cu
        _, counts = np.unique(ids, return_counts=True)
        print(f"  CUs used {len(counts)}, blocks/CU max {counts.max()} median {np.median(counts)}; "
              f"XCC histogram {np.bincount(xcc, minlength=8).tolist()}")


if __name__ == "__main__":
    main()
