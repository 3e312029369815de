"""Phase timeline of k_env (env tick + replay push + bookkeeping) per env block, from the
diagnostic library's PM_ENV_STAMP stamps (s_memrealtime, 10 ns; each stamp first drains the wave's
memory operations only at the end: a phase is the time the wave's instruction stream takes to get
through it, waits the compiler placed in it included).

    make -C pingpong-selfplay-ai_amd/csrc diag && python tools/env_blocks.py

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

PHASES = ["begin", "loads issued + speculative draws (+ act tiles, fused)", "state wait + tick + obs", "bookkeeping + replay/state stores",
          "LDS staging + barrier", "partials + opponent lists", "obs stores + drain of all stores (end)"]


def main():
    import bench
    from pongmi import _lib
    from pongmi.selfplay import SelfPlayLearner
    lib = _lib.load()
    lib.pm_diag_read_env.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    n = 65536
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    L = SelfPlayLearner(bench.ENV_KW, n, sdB, sdA, pool, batch=256, memory_size=1_000_000, epsilon=0.08, seed=7)
    for _ in range(40):
        L.step()
    torch.cuda.synchronize()
    nb = (n + 255) // 256
    buf = (ctypes.c_uint64 * (8 * 1024))()
    blk = (ctypes.c_uint64 * (8 * 4096))()
    sfb = 64 if os.environ.get("PONGMI_SFB") == "64" else 32  # samples per k_actenv sampler block
    nsb = (256 + sfb - 1) // sfb
    acc, samp, staged = [], [], []
    for _ in range(20):
        if L.overlap:  # the production step's launches, read right after the fused act + env kernel
            L.actenv()
        else:
            L.step()
        torch.cuda.synchronize()
        lib.pm_diag_read_env(buf)
        full = np.array(buf[:], dtype=np.int64).reshape(8, 1024)
        a = full[:7, :nb]
        acc.append(a)
        if L.overlap:
            staged.append((full[7, :nb] - a[0]) * 0.01)
        if L.overlap:
            lib.pm_diag_read_blk(blk)
            b = np.array(blk[:], dtype=np.int64).reshape(8, 4096)[:, :nsb]
            samp.append((b - a[0].min()) * 0.01)
            L.learn(act_next=True)
            L.apply()
    spans, deltas = [], [[] for _ in PHASES]
    for a in acc:
        t0 = a[0].min()
        spans.append((a[6].max() - t0) * 0.01)
        deltas[0].extend((a[0] - t0) * 0.01)
        for k in range(1, 7):
            deltas[k].extend((a[k] - a[k - 1]) * 0.01)
    print(f"k_env env blocks: {nb}; span first begin -> last end: median {np.median(spans):.2f} us")
    for k, name in enumerate(PHASES):
        v = np.array(deltas[k])
        label = "begin offset" if k == 0 else name
        print(f"  {label:44s} p50 {np.percentile(v, 50):6.2f}  p90 {np.percentile(v, 90):6.2f}  max {v.max():6.2f} us")
    if staged:
        v = np.concatenate(staged)
        print(f"  (fused) begin -> loads landed + weights staged  p50 {np.percentile(v, 50):6.2f}  p90 "
              f"{np.percentile(v, 90):6.2f}  max {v.max():6.2f} us")
    if samp:
        s = np.stack(samp)  # [run][slot][block]
        q = lambda v: " ".join(f"{x:6.2f}" for x in np.percentile(v, [0, 50, 90, 100]))  # noqa: E731
        print(f"k_actenv sampler+forward blocks ({nsb}), times from the first env block's begin (min p50 p90 max):")
        print(f"  begin {q(s[:, 0])} | level2 {q(s[:, 4])} | level1 {q(s[:, 5])} | leaves {q(s[:, 6])} | "
              f"sampled {q(s[:, 1])} | end {q(s[:, 2])}")


if __name__ == "__main__":
    main()
