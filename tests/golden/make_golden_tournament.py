#!/usr/bin/env python3
"""Golden fixture for the round-robin tournament (tests/test_round_robin.py:117-386), produced by
running the REFERENCE's env and model modules in this container:

    python -B tests/golden/make_golden_tournament.py

Participants (checkpoints loaded with torch.load(weights_only=True)):
  RNN_Gen1   checkpoints_rnn/rnn_agent_1.pth      QNetRNN
  RNN_Soul3  checkpoints_rnn/rnn_pong_soul_3.pth  QNetRNN
  Legacy4_12 checkpoints/model4-12.pth            QNet, legacy fc.* keys (mapped as :157-168)
  Noisy5_5   checkpoints/model5-5_fault.pth       QNet, dueling NoisyNet keys
  Bot        HardcodedBallFollower (:207-228)
The model loading (:134-185), action selection (:190-235) and match loop (:283-330) are restated
below over the reference's PongEnv2P / QNet / QNetRNN, with the env of config.yaml and
random.seed(SEED) before the first match. Writes tournament.npz: the checkpoint dicts' state
tensors (the tournament loads them itself; RNN_Soul3's are rnn.npz's params.*), the pair order and
per-episode (score_A, score_B).
"""
import os
import random
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import REF  # noqa: E402  (installs the gym / pygame stubs, puts REF on sys.path)

import torch  # noqa: E402
import yaml  # noqa: E402
from envs.my_pong_env_2p import PongEnv2P  # noqa: E402
from models.qnet import QNet  # noqa: E402
from models.qnet_rnn import QNetRNN  # noqa: E402

SEED, EPISODES = 20250806, 10
PARTICIPANTS = [
    ("RNN_Gen1", "checkpoints_rnn/rnn_agent_1.pth", "QNetRNN"),
    ("RNN_Soul3", "checkpoints_rnn/rnn_pong_soul_3.pth", "QNetRNN"),
    ("Legacy4_12", "checkpoints/model4-12.pth", "QNet"),
    ("Noisy5_5", "checkpoints/model5-5_fault.pth", "QNet"),
    ("Bot", "N/A", "HardcodedBallFollower"),
]
KEYS = ["modelB_state", "modelA_state", "modelB", "modelA", "model", "state_dict"]


def state_of(ckpt):
    for k in KEYS:
        if k in ckpt:
            return ckpt[k]
    return ckpt


def load(path, typ):
    if typ == "HardcodedBallFollower":
        return None, {}
    sd = state_of(torch.load(os.path.join(REF, path), map_location="cpu", weights_only=True))
    if typ == "QNet":
        net = QNet(7, 3)
        if any(k.startswith(("features.", "fc_V.", "fc_A.")) for k in sd):
            net.load_state_dict(sd, strict=True)
        else:  # legacy fc.* -> dueling mu (the reference's mapping)
            m = {}
            for k, v in sd.items():
                if k.startswith("fc.0."):
                    m[k.replace("fc.0.", "features.0.")] = v
                elif k.startswith("fc.2."):
                    m[k.replace("fc.2.", "features.2.")] = v
            w4, b4 = sd["fc.4.weight"], sd["fc.4.bias"]
            m["fc_A.weight_mu"], m["fc_A.bias_mu"] = w4, b4
            m["fc_V.weight_mu"], m["fc_V.bias_mu"] = w4.mean(dim=0, keepdim=True), b4.mean().unsqueeze(0)
            net.load_state_dict(m, strict=False)
    else:
        net = QNetRNN(7, 3)
        net.load_state_dict(sd)
    net.eval()
    net.reset_noise()
    return net, sd


def act(obs, net, typ, hidden):
    with torch.no_grad():
        if typ == "QNetRNN":
            q, hidden = net(torch.tensor(obs, dtype=torch.float32).unsqueeze(0).unsqueeze(0), hidden)
            return int(q.argmax(1).item()), hidden
        if typ == "QNet":
            return int(net(torch.tensor(obs, dtype=torch.float32).unsqueeze(0)).argmax(1).item()), None
        ball_x, my_x, tol = obs[0], obs[4], 0.01
        return (0 if ball_x < my_x - tol else 2 if ball_x > my_x + tol else 1), None


def main():
    torch.manual_seed(0)
    with open(os.path.join(REF, "config.yaml")) as f:
        env_params = yaml.safe_load(f)["env"]
    env_params["enable_render"] = False
    env = PongEnv2P(**env_params)
    nets, out = [], {}
    for i, (name, path, typ) in enumerate(PARTICIPANTS):
        net, sd = load(path, typ)
        nets.append(net)
        if name != "RNN_Soul3":  # its state dict is rnn.npz's params.* (the same modelB_state)
            for k, v in sd.items():
                out[f"sd{i}.{k}"] = v.numpy()
    random.seed(SEED)
    pairs, scores = [], []
    for i in range(len(PARTICIPANTS)):
        for j in range(i + 1, len(PARTICIPANTS)):
            pairs.append((i, j))
            for _ in range(EPISODES):
                oA, oB = env.reset()
                done = False
                hA = nets[i].init_hidden(1, "cpu") if PARTICIPANTS[i][2] == "QNetRNN" else None
                hB = nets[j].init_hidden(1, "cpu") if PARTICIPANTS[j][2] == "QNetRNN" else None
                while not done:
                    aA, hA = act(oA, nets[i], PARTICIPANTS[i][2], hA)
                    aB, hB = act(oB, nets[j], PARTICIPANTS[j][2], hB)
                    (oA, oB), _, done, _ = env.step(aA, aB)
                scores.append((env.scoreA, env.scoreB))
    out["pairs"] = np.array(pairs, np.int32)
    out["scores"] = np.array(scores, np.int32).reshape(len(pairs), EPISODES, 2)
    out["seed"] = np.array(SEED)
    out["names"] = np.array([p[0] for p in PARTICIPANTS])
    out["types"] = np.array([p[2] for p in PARTICIPANTS])
    out["random_state_after"] = np.array(random.random())  # one draw past the tournament's consumption
    np.savez_compressed(os.path.join(HERE, "tournament.npz"), **out)
    s = out["scores"]
    print("wrote tournament.npz", sum(v.nbytes for v in out.values()), "bytes;",
          "A wins", int((s[..., 0] > s[..., 1]).sum()), "B wins", int((s[..., 1] > s[..., 0]).sum()))


if __name__ == "__main__":
    main()
