"""Phase timeline of one vector step from the diagnostic library's in-kernel stamps.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/stamps.py [--steps 20]

Thread 0 of block 0 of each learner kernel records s_memrealtime (100 MHz) at phase boundaries
(PM_STAMP in pm_selfplay.hip); this prints the median time of every stamp relative to the start of
the step's first kernel (k_actenv's first env block in the fused step, k_act_sp's first act block in
the plain one), i.e. the critical path through act + env (+ PER sample blocks) -> learn.
Diagnostic only (libpongmi_diag.so, never the product library).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["PONGMI_LIB"] = os.environ.get(  # PONGMI_DIAG_LIB: another diagnostic build (e.g. -DPM_DIAG_NOWAIT)
    "PONGMI_DIAG_LIB", os.path.join(ROOT, "pingpong-selfplay-ai_amd", "pongmi", "libpongmi_diag.so"))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

NAMES = {
    70: "act start (1st act blk)", 64: "sample start", 65: "sample blk0 end", 72: "env start (1st env blk)",
    0: "learn start", 30: "ph0 issued", 31: "ph0 idx/isw in", 32: "ph0 hfeat in", 33: "ph0 trans in",
    1: "learn loads", 2: "learn fwd (MFMA)", 3: "learn td/loss", 4: "learn scatter+grad",
    8: "ph4 grads out w0", 9: "ph4 grads out w15", 10: "ph4 scatter subs w0", 11: "ph4 scatter subs w15",
    12: "ph4 push subs w0", 13: "ph4 push subs w15", 14: "ph4 edges w0", 15: "ph4 edges w15",
    35: "ph0 before prologue", 34: "ph0 after prologue", 40: "ph0 w0 loads landed",
    41: "ph0 w4 loads landed", 42: "ph0 w8 loads landed", 43: "ph0 w15 loads landed",
    50: "push blk start", 51: "push blk loads", 52: "push blk fwd done", 53: "push blk stores drained",
    16: "ph0 w0: idx + ctrl in", 17: "ph0 w0: partials in", 18: "ph0 w0: isw in", 19: "ph0 w15 at DMA issue",
    54: "learn push flag seen", 36: "ph1 push token polled (t0)", 37: "ph1 eps-decay pow done (t1023)", 55: "tree blk start", 56: "tree blk prefetch issued",
    57: "tree blk granules + DMA in", 58: "tree blk level 1 done", 59: "tree blk level 2 done",
    60: "tree blk winners + pval (t0)", 61: "tree blk level-1 sums (t0)", 62: "tree blk pushed subs (t0)",
    63: "tree blk chunk slots (t0)", 66: "learn launch: side-A act blocks end (max)",
    67: "learn launch: feature blocks end (max)",
    5: "learn tree level1", 6: "learn tree level2", 20: "apply adam", 21: "apply derive", 7: "learn end",
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--arenas", type=int, default=65536)
    ap.add_argument("--plain", action="store_true", help="the plain step (k_learn without side blocks)")
    args = ap.parse_args()
    import bench
    from pongmi import _lib
    from pongmi.selfplay import SelfPlayLearner
    lib = _lib.load()
    lib.pm_diag_read.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32]
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    L = SelfPlayLearner(bench.ENV_KW, args.arenas, sdB, sdA, pool, batch=256, memory_size=1_000_000,
                        epsilon=0.08, seed=7, overlap=not args.plain)
    for _ in range(args.warmup):
        L.step()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 256)()
    rows = []
    for _ in range(args.steps):
        lib.pm_diag_clear()
        L.step()
        torch.cuda.synchronize()
        lib.pm_diag_read(buf, 256)
        v = np.array(buf[:], dtype=np.int64)
        rows.append(v)
    a = np.stack(rows)
    base = a[:, 70:71] if (a[:, 70] != 0).all() else a[:, 72:73]
    rel = (a - base) * 0.01  # 100 MHz ticks -> us
    for slot in sorted(NAMES, key=lambda s: np.median(rel[:, s])):
        if (a[:, slot] == 0).any():
            continue
        print(f"{slot:3d} {NAMES[slot]:22s} {np.median(rel[:, slot]):9.2f} us  (min {rel[:, slot].min():8.2f})")


if __name__ == "__main__":
    main()
