"""Time the K5 QNetRNN kernels on the device: pm_rnn_q and the fused two-player pm_rnn_act at
65536 arenas (pool of 8 opponents + the learner). Prints one JSON line per kernel with the
arena-steps/s and the MFMA-rate fraction (exact-f32 MFMA peak from the microarch guide)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "pingpong-selfplay-ai_amd"))

# multiply-adds per arena-step: 7x64 (+bias row) + 64x128 + 256x512 + 128x128 + 128x4
MAC = 8 * 64 + 64 * 128 + 256 * 512 + 128 * 128 + 128 * 4
F32_MFMA_PEAK = 157.3e12  # FLOP/s, dense fp32 MFMA (MI355X_MICROARCH.md)


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    from models.qnet_rnn import QNetRNN
    from pongmi import _lib, rnn
    torch.manual_seed(0)
    nets = [QNetRNN(7, 3) for _ in range(a.pool + 1)]
    w = rnn.fold(torch.stack([rnn.pack_state_dict(m.state_dict()) for m in nets]), _lib.PM_FOLD_TRAIN)
    n = a.n
    obsA = torch.rand(n, 7, device="cuda")
    obsB = torch.rand(n, 7, device="cuda")
    opp = torch.randint(0, a.pool + 1, (n,), device="cuda", dtype=torch.int32)
    h, c = rnn.init_state(n)
    stA, stB = rnn.init_state(n), rnn.init_state(n)
    t_q = timed(lambda: rnn.q_step(w[0], obsB, h, c), a.iters)
    chunk1 = min(2048, max(256, (2 * n // (a.pool + 1) + 255) // 256 * 256))
    t_act = timed(lambda: rnn.act(w[1:], opp % a.pool, w[0], obsA, obsB, stA, stB, epsilon=0.1, chunk1=chunk1),
                  a.iters)
    for name, t, rows in (("pm_rnn_q", t_q, n), ("pm_rnn_act", t_act, 2 * n)):
        fl = 2.0 * MAC * rows / t
        print(json.dumps({"kernel": name, "arenas": n, "rows": rows, "us": round(t * 1e6, 1),
                          "rows_per_s": rows / t, "tflops": fl / 1e12, "mfma_frac": fl / F32_MFMA_PEAK}))


if __name__ == "__main__":
    main()
