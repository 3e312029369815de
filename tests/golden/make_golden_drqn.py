#!/usr/bin/env python3
"""Golden fixtures for the DRQN update (train_step_rnn, scripts/train_rnn_iterative.py:400-531),
produced with the REFERENCE's QNetRNN module and torch autograd.

Run only in the build container (the reference does not exist on the GPU box):

    python -B tests/golden/make_golden_drqn.py

modelB = QNetRNN with rnn.npz's params (checkpoints_rnn/rnn_pong_soul_3.pth modelB_state), train mode
(NoisyLinear uses the stored epsilon buffers; train_step_rnn does not reset noise). targetB = a copy
of modelB in eval mode (:263-265, :336-338). Adam(modelB.parameters(), lr=1e-4) (:335), gamma 0.99,
clip_grad_norm_(1.0) (:515). Three updates on three synthetic [64, 8] sequence batches; the update
body below restates :424-517 (zero initial state; Q_B(obs) last step gathered at the last action;
double-DQN target with modelB / targetB on next_obs; smooth_l1_loss; backward; clip; step).

Writes drqn.npz:
  b{k}_obs [64,8,7], b{k}_act [64,8] int64, b{k}_rew [64,8], b{k}_next [64,8,7], b{k}_done [64,8] bool
  u0_q, u0_target, u0_loss, u0_norm     first update: Q(s,a), TD target, loss, pre-clip total norm
  u0_grad.<name>                        first update: gradients of every parameter (pre-clip)
  u{k}_loss, u{k}_norm                  updates 1, 2
  final_sub.<name>                      parameters after 3 updates, every 8th element (flattened)
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.dont_write_bytecode = True
REF = os.environ.get("PONG_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
GAMMA, LR, CLIP, BATCH, T = 0.99, 1e-4, 1.0, 64, 8


def batch(rng):
    obs = rng.uniform(0, 1, (BATCH, T + 1, 7)).astype(np.float32)
    obs[..., 2:4] = rng.uniform(-0.08, 0.08, (BATCH, T + 1, 2))
    obs[..., 6] = rng.uniform(-5, 5, (BATCH, T + 1))
    act = rng.integers(0, 3, (BATCH, T)).astype(np.int64)
    rew = rng.choice(np.array([-1.0, 0.0, 1.0], np.float32), (BATCH, T), p=[0.1, 0.8, 0.1]).astype(np.float32)
    done = rng.random((BATCH, T)) < 0.25
    return obs[:, :T].copy(), act, rew, obs[:, 1:].copy(), done


def update(modelB, targetB, opt, b):
    obs, act, rew, nxt, done = (torch.from_numpy(x) for x in b)
    zB = modelB.init_hidden(BATCH, "cpu")
    zT = targetB.init_hidden(BATCH, "cpu")
    qB, _ = modelB(obs, zB)
    q = qB.gather(1, act[:, -1].unsqueeze(1)).squeeze(1)
    with torch.no_grad():
        a_star = modelB(nxt, zT)[0].argmax(dim=1, keepdim=True)
        qT = targetB(nxt, zT)[0].gather(1, a_star).squeeze(1)
        y = rew[:, -1] + GAMMA * qT * (~done[:, -1])
    loss = F.smooth_l1_loss(q, y)
    opt.zero_grad()
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in modelB.named_parameters()}
    norm = torch.nn.utils.clip_grad_norm_(modelB.parameters(), max_norm=CLIP)
    opt.step()
    return q.detach(), y, loss.detach(), norm.detach(), grads


def main():
    sys.path.insert(0, REF)
    from models.qnet_rnn import QNetRNN  # the reference module
    torch.manual_seed(0)
    g = dict(np.load(os.path.join(OUT, "rnn.npz")))
    sd = {k[7:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("params.")}
    modelB = QNetRNN(7, 3)
    modelB.load_state_dict(sd)
    modelB.train()
    targetB = QNetRNN(7, 3)
    targetB.load_state_dict(modelB.state_dict())
    targetB.eval()
    opt = torch.optim.Adam(modelB.parameters(), lr=LR)
    rng = np.random.default_rng(2024)
    out = {}
    for k in range(3):
        b = batch(rng)
        for name, x in zip(("obs", "act", "rew", "next", "done"), b):
            out[f"b{k}_{name}"] = x
        q, y, loss, norm, grads = update(modelB, targetB, opt, b)
        out[f"u{k}_loss"] = loss.numpy()
        out[f"u{k}_norm"] = norm.numpy()
        if k == 0:
            out["u0_q"], out["u0_target"] = q.numpy(), y.numpy()
            for n, v in grads.items():
                out[f"u0_grad.{n}"] = v.numpy()
    for n, p in modelB.named_parameters():
        out[f"final_sub.{n}"] = p.detach().reshape(-1)[::8].numpy().copy()
    np.savez_compressed(os.path.join(OUT, "drqn.npz"), **out)
    print("wrote", os.path.join(OUT, "drqn.npz"), sum(v.nbytes for v in out.values()), "bytes",
          "losses", [float(out[f"u{k}_loss"]) for k in range(3)], "norms", [float(out[f"u{k}_norm"]) for k in range(3)])


if __name__ == "__main__":
    main()
