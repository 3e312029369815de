"""Phase timeline of one DRQN update (diagnostic library): s_memrealtime stamps (100 MHz) of the
embed / recurrence / weight-gradient kernels, relative to k_dq_embed's start.

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/drqn_stamps.py
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

NAMES = {220: "embed start", 222: "embed block 0 end (wave 4)", 1: "recur obs WG start", 111: "recur target WG 0 start"}
for t in range(20):
    NAMES[10 + t] = f"  obs fwd step {t} done (barrier)"
    NAMES[120 + t] = f"  tgt fwd step {t} done (barrier)"
    NAMES[90 + t] = f"  obs bwd step {t}: dh_(t-1) reduced"
for t in range(20):
    NAMES[180 + t] = f"  dF2 trailer step {t}: dF2 reduced"
NAMES.update({228: "embed b0: first loads landed (diag drain)", 227: "embed b0: after setup", 223: "embed b0: F1/F2 done (thread 0)", 224: "embed b0: F2 barrier", 225: "embed b0: Zx MFMAs done", 226: "embed b0: halves barrier", 8: "dF2 trailer 0 start", 7: "dF2 trailer 0 end", 50: "obs heads: Q formed", 150: "target WG 0: Q published", 51: "obs: target Q gathered, loss",
              52: "obs: dh_T reduced", 2: "recur obs WG end", 210: "wgrad A start", 211: "wgrad A tile done",
              200: "wgrad B start", 201: "wgrad B dF2 done", 204: "wgrad B dF1 done", 206: "wgrad B ticket",
              207: "wgrad last tile: reduce start", 208: "wgrad last tile: reduce end"})


def main():
    import bench
    from pongmi import _lib
    from pongmi.drqn import DRQNLearner
    lib = _lib.load()
    lib.pm_diag_read_drqn.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    B, T = 64, 8
    L = DRQNLearner(bench.synthetic_rnn(1), bench.synthetic_rnn(2), batch=B, T=T)
    g = torch.Generator().manual_seed(0)
    L.load_batch(torch.rand(B, T, 7, generator=g), torch.randint(0, 3, (B, T), generator=g),
                 torch.randint(-1, 2, (B, T), generator=g).float(), torch.rand(B, T, 7, generator=g),
                 torch.rand(B, T, generator=g) < 0.1)
    for _ in range(10):
        L.update()
    torch.cuda.synchronize()
    buf = (ctypes.c_uint64 * 256)()
    rows = []
    for _ in range(5):
        lib.pm_diag_clear_drqn()
        L.update()
        torch.cuda.synchronize()
        lib.pm_diag_read_drqn(buf)
        rows.append(np.array(buf[:], dtype=np.int64))
    r = np.median(np.stack(rows), axis=0)
    t0 = r[220]
    for k in sorted(NAMES, key=lambda k: r[k] if r[k] else 1e30):
        if r[k]:
            print(f"{NAMES[k]:40s} {(r[k] - t0) / 100.0:9.2f} us")
    print("status", L.stats()["status"])


if __name__ == "__main__":
    main()
