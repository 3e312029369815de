"""Time the DRQN update alone (pm_drqn_update: 5 launches) at batch 64 x T 8, HIP events over
back-to-back updates on one stream, and the persistent recurrence by its own dispatch."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from bench import synthetic_rnn  # noqa: E402
from pongmi import _lib  # noqa: E402
from pongmi.drqn import DRQNLearner  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--T", type=int, default=8)
ap.add_argument("--n", type=int, default=200)
args = ap.parse_args()
B, T = args.batch, args.T
L = DRQNLearner(synthetic_rnn(1), synthetic_rnn(2), batch=B, T=T)
g = torch.Generator().manual_seed(0)
L.load_batch(torch.rand(B, T, 7, generator=g), torch.randint(0, 3, (B, T), generator=g),
             torch.randint(-1, 2, (B, T), generator=g).float(), torch.rand(B, T, 7, generator=g),
             torch.rand(B, T, generator=g) < 0.1)
for _ in range(20):
    L.update()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(args.n):
    L.update()
e1.record()
e1.synchronize()
us = e0.elapsed_time(e1) * 1e3 / args.n
rec = []
for _ in range(20):
    _lib.timer_arm(_lib.PM_TIMER_DRQN)
    L.update()
rec = [_lib.timer_read(_lib.PM_TIMER_DRQN) * 1e6 for _ in range(20)]
st = L.stats()
print(json.dumps({"batch": B, "T": T, "update_us": round(us, 2), "recur_us": round(sum(rec) / len(rec), 2),
                  "loss": st["loss"], "norm": st["norm"], "status": st["status"]}), flush=True)
