"""Extract the state dicts of the reference tournament's six QNetRNN checkpoints
(tests/test_round_robin.py USER_CONFIG, results/summary_ranking_20250806_213819.csv) into
tests/golden/_local/tournament_models.npz (git-ignored; travels to the GPU box with the working
tree for tools/tournament_replication.py). Run in the build container only:

    python -B tools/extract_tournament_weights.py
"""
import os

import numpy as np
import torch

REF = os.environ.get("PONG_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "_local")
MODELS = [("RNN_Gen1", "checkpoints_rnn/rnn_agent_1.pth"), ("RNN_Gen2", "checkpoints_rnn/rnn_agent_2.pth"),
          ("RNN_Gen3", "checkpoints_rnn/rnn_agent_3.pth"), ("RNN_Gen4", "checkpoints_rnn/rnn_agent_4.pth"),
          ("RNN_Gen5", "checkpoints_rnn/rnn_pong_soul_1.pth"), ("RNN_Gen6", "checkpoints_rnn/rnn_pong_soul_2.pth")]
KEYS = ["modelB_state", "modelA_state", "modelB", "modelA", "model", "state_dict"]


def main():
    os.makedirs(OUT, exist_ok=True)
    out = {}
    for name, path in MODELS:
        cp = torch.load(os.path.join(REF, path), map_location="cpu", weights_only=True)
        sd = next(cp[k] for k in KEYS if k in cp)
        for k, v in sd.items():
            out[f"{name}.{k}"] = v.numpy()
    np.savez(os.path.join(OUT, "tournament_models.npz"), **out)
    print("wrote", os.path.join(OUT, "tournament_models.npz"))


if __name__ == "__main__":
    main()
