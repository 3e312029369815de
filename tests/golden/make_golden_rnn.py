#!/usr/bin/env python3
"""Golden fixtures for the QNetRNN path, produced by running the REFERENCE itself.

Run only in the build container (the reference does not exist on the GPU box):

    python -B tests/golden/make_golden_rnn.py

Imports the reference's models/qnet_rnn.py (torch only) and loads
checkpoints_rnn/rnn_pong_soul_3.pth with torch.load(weights_only=True). Writes inputs and the
reference's outputs as rnn.npz:

  act_*   one acting step, x [64, 1, 7] with non-zero (h, c) [1, 64, 128] (models/qnet_rnn.py:107-144),
          train mode (NoisyLinear uses the checkpoint's epsilon buffers) and eval mode (mu)
  seq_*   T = 8 sequences from zero hidden state (train_rnn_iterative.py:424-426, :449), both modes
  roll_*  12 consecutive acting steps of 16 arenas, hidden state carried (select_action_for_model,
          train_rnn_iterative.py:371-389, greedy branch without reset_noise)
  params  the modelB state_dict (float32)
"""
import os
import sys

import numpy as np
import torch

sys.dont_write_bytecode = True
REF = os.environ.get("PONG_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    sys.path.insert(0, REF)
    from models.qnet_rnn import QNetRNN  # the reference module
    torch.manual_seed(0)
    cp = torch.load(os.path.join(REF, "checkpoints_rnn", "rnn_pong_soul_3.pth"), map_location="cpu", weights_only=True)
    sd = cp["modelB_state"]
    net = QNetRNN(7, 3)
    net.load_state_dict(sd)
    out = {f"params.{k}": v.numpy().astype(np.float32) for k, v in sd.items()}
    rng = np.random.default_rng(5)

    def obs(*shape):  # plausible observations: positions in [0,1], velocities small, spin in [-5,5]
        x = rng.uniform(0, 1, shape + (7,)).astype(np.float32)
        x[..., 2:4] = rng.uniform(-0.08, 0.08, shape + (2,))
        x[..., 6] = rng.uniform(-5, 5, shape)
        return x.astype(np.float32)

    with torch.no_grad():
        # one acting step with a warm hidden state
        x = obs(64, 1)
        h0 = torch.from_numpy(rng.normal(0, 0.3, (1, 64, 128)).astype(np.float32))
        c0 = torch.from_numpy(rng.normal(0, 0.6, (1, 64, 128)).astype(np.float32))
        out["act_x"], out["act_h0"], out["act_c0"] = x, h0.numpy(), c0.numpy()
        for mode in ("train", "eval"):
            net.train(mode == "train")
            q, (h1, c1) = net(torch.from_numpy(x), (h0, c0))
            out[f"act_q_{mode}"], out[f"act_h1_{mode}"], out[f"act_c1_{mode}"] = q.numpy(), h1.numpy(), c1.numpy()
        # T = 8 sequences from zero state (the DRQN update's forward)
        xs = obs(16, 8)
        out["seq_x"] = xs
        for mode in ("train", "eval"):
            net.train(mode == "train")
            q, (h, c) = net(torch.from_numpy(xs), net.init_hidden(16, "cpu"))
            out[f"seq_q_{mode}"], out[f"seq_h_{mode}"], out[f"seq_c_{mode}"] = q.numpy(), h.numpy(), c.numpy()
        # 12 acting steps, hidden state carried
        net.train(True)
        xr = obs(12, 16)
        h, c = net.init_hidden(16, "cpu")
        qs = []
        for t in range(12):
            q, (h, c) = net(torch.from_numpy(xr[t]).unsqueeze(1), (h, c))
            qs.append(q.numpy())
        out["roll_x"], out["roll_q"], out["roll_h"], out["roll_c"] = xr, np.stack(qs), h.numpy(), c.numpy()
    np.savez_compressed(os.path.join(OUT, "rnn.npz"), **out)
    print("wrote", os.path.join(OUT, "rnn.npz"), sum(v.nbytes for v in out.values()), "bytes")


if __name__ == "__main__":
    main()
