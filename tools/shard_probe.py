#!/usr/bin/env python3
"""Sharded-step probe on ONE device: what the N > 1 bench step costs besides the collective's wire
time. Per configuration, wall time per vector step over K steps and the host time spent issuing them.

    python tools/shard_probe.py [--steps 300]

  fused     world 1: the production two-launch step (k_actenv, k_learn + Adam)
  split     the sharded launch sequence (k_actenv, k_learn, k_adam), no collective
  torch     world-2 arithmetic: the Python sequence + torch.distributed.all_reduce on a 1-rank nccl
            (RCCL) group
  native    the library's own RCCL communicator: one C-ABI call per step (pm_selfplay_step_sharded)
            with ncclAllReduce on the learner's stream
The 1-rank group has no wire time: the difference torch - split is the collective's launch path.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import ENV_KW, synthetic_qnet  # noqa: E402


def run(kind, steps, dist):
    from pongmi.dist import NativeComm
    from pongmi.selfplay import SelfPlayLearner
    world, fuse, allreduce, comm = 1, True, None, None
    if kind == "split":  # world-1 learner with the sharded launch sequence, no collective
        fuse = False
    elif kind == "torch":  # world-2 arithmetic, Python sequence + torch all_reduce on the 1-rank group
        world, fuse, allreduce = 2, False, (lambda t: dist.all_reduce(t))
    elif kind == "native":  # one library call per step, ncclAllReduce in the learner's stream
        fuse, comm = False, NativeComm()
        allreduce = comm
    L = SelfPlayLearner(ENV_KW, 65536, synthetic_qnet(1), synthetic_qnet(2), [synthetic_qnet(100 + k) for k in range(8)],
                        batch=256, memory_size=1_000_000, epsilon=0.08, seed=7, world=world, rank=0,
                        allreduce=allreduce, fuse_apply=fuse)
    for _ in range(30):
        L.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        L.step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return {"kind": kind, "us_per_step": round((t2 - t0) / steps * 1e6, 2),
            "host_us_per_step": round((t1 - t0) / steps * 1e6, 2), "steps": steps,
            "train_steps": L.counters()["train_steps"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    a = ap.parse_args()
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    for kind in ("fused", "split", "torch", "native"):
        print(json.dumps(run(kind, a.steps, dist)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
