"""Match megakernel (K8) vs the stepped evaluator loop: wall time and env-steps/s for greedy
episodes between random-init QNets at evaluator and tournament sizes.

    python tools/play_bench.py [--episodes 1000 21000 65536] [--json out.json]
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pingpong-selfplay-ai_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1,
              friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
              ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1, speed_increment=0.1)  # config.yaml


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, nargs="+", default=[1000, 21000, 65536])
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--stepped-max", type=int, default=21000, help="largest size also timed on the stepped loop")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    from models.qnet import QNet
    from pongmi import _lib
    from pongmi.env import draw_serve, env_config
    from pongmi.evaluate import folded_weights, run_episodes, run_episodes_stepped
    nets = []
    for i in range(args.pool + 1):
        torch.manual_seed(i)
        nets.append(folded_weights((QNet(7, 3).state_dict(), _lib.PM_FOLD_EVAL), "cuda"))
    w = torch.stack(nets)
    cfg = env_config(**ENV_KW)
    rows = []
    for E in args.episodes:
        rng = random.Random(E)
        serves = np.array([draw_serve(rng, cfg) for _ in range(E)], np.float64)
        opp = np.random.default_rng(E).integers(0, args.pool, E).astype(np.int32)
        res = {}
        for name, fn in (("megakernel", run_episodes), ("stepped", run_episodes_stepped)):
            if name == "stepped" and E > args.stepped_max:
                continue
            fn(ENV_KW, w[:args.pool], opp[:256], w[args.pool], serves[:256])  # warm up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            wins, length = fn(ENV_KW, w[:args.pool], opp, w[args.pool], serves)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[name] = dict(seconds=round(dt, 5), env_steps=int(length.sum()), max_len=int(length.max()),
                             env_steps_per_s=round(float(length.sum()) / dt, 1), win_rate=float(wins.mean()))
        if "stepped" in res:
            res["speedup"] = round(res["stepped"]["seconds"] / res["megakernel"]["seconds"], 2)
        rows.append({"episodes": E, "pool": args.pool, **res})
        print(json.dumps(rows[-1]), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
