"""How well-conditioned each DRQN fixture update is in float32: for every update
dumped by tests/test_gpu_drqn.py (PONGMI_DRQN_DUMP=<dir>: the device's pre-update parameters and its
gradient), the float64 oracle's gradient at those parameters against (a) the device's gradient and
(b) the reference's own float32 autograd (tests/test_gpu_drqn.py::ref32_grads: torch on the CPU, the
reference module tree), per tensor as max |error| / max |g|; plus the closest argmax margin of
Q_B(next) and the smallest | |d| - 1 | of the Huber loss (the loss's discrete decisions).

    python tools/drqn_conditioning.py gpurun_out/r6c_dump
"""
import glob
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pingpong-selfplay-ai_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402

import test_gpu_drqn as T  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main(d):
    gr = dict(np.load(os.path.join(ROOT, "tests", "golden", "rnn.npz")))
    gd = dict(np.load(os.path.join(ROOT, "tests", "golden", "drqn.npz")))
    tsd = {k[7:]: v.astype(np.float64) for k, v in gr.items() if k.startswith("params.")}
    for f in sorted(glob.glob(os.path.join(d, "drqn_u*.npz"))):
        u = int(os.path.basename(f)[6:-4])
        z = dict(np.load(f))
        p = {k[2:]: v.astype(np.float64) for k, v in z.items() if k.startswith("p.")}
        g = {k[2:]: v for k, v in z.items() if k.startswith("g.")}
        batch = T._batch(gd, u)
        info = orc.drqn_grads(p, tsd, *batch)
        r32 = T.ref32_grads(p, tsd, *batch)
        obs, act, rew, nxt, done = batch
        eB = orc.rnn_effective(p, True)
        zz = np.zeros((obs.shape[0], 128))
        qn = np.sort(orc.rnn_forward(eB, nxt, zz, zz)[0], 1)
        d = info["q"] - info["y"]
        print(f"update {u}: loss {info['loss']:.6f}; closest argmax margin of Q_B(next) {float((qn[:, 2] - qn[:, 1]).min()):.2e}; "
              f"min | |d| - 1 | {float(np.abs(np.abs(d) - 1).min()):.3f}")
        print(f"  {'tensor':34s} {'device':>10s} {'ref f32':>10s}   (max |x - float64| / max |g|)")
        for k, r in info["grads"].items():
            m = np.abs(r).max()
            print(f"  {k:34s} {np.abs(g[k] - r).max() / m:10.2e} {np.abs(r32[k] - r).max() / m:10.2e}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "r6c_dump"))
