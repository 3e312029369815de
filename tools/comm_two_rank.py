#!/usr/bin/env python3
"""Two ranks through libpongmi's RCCL communicator (pongmi.dist.NativeComm): the in-stream all-reduce
sums across processes, and two sharded DQN learners (world 2, rank-specific arenas) stay bitwise
identical through pm_selfplay_step_sharded. The id broadcast and the checks run over a gloo group.
Each rank takes device local_rank % device_count: RCCL rejects two ranks on one GPU
(ncclCommInitRank: invalid usage, measured on the 1-GPU box; both ranks raise, nothing hangs), so
this needs a box with two GPUs.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \\
        tools/comm_two_rank.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bench import ENV_KW, synthetic_qnet  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
    from pongmi.dist import NativeComm
    from pongmi.selfplay import SelfPlayLearner
    comm = NativeComm()
    x = torch.full((4096,), float(rank + 1), device="cuda")
    comm(x)
    torch.cuda.synchronize()
    ok_sum = bool(torch.all(x == world * (world + 1) / 2).item())
    L = SelfPlayLearner(ENV_KW, 8192, synthetic_qnet(1), synthetic_qnet(2), [synthetic_qnet(100 + k) for k in range(4)],
                        batch=256, memory_size=65536, epsilon=0.3, seed=7, rank=rank, world=world, allreduce=comm)
    for _ in range(60):
        L.step()
    torch.cuda.synchronize()
    p = L.paramsB.cpu()
    ps = [torch.zeros_like(p) for _ in range(world)]
    dist.all_gather(ps, p)
    c = L.counters()
    same = all(torch.equal(ps[0], q) for q in ps)
    if rank == 0:
        print({"allreduce_sum_ok": ok_sum, "replicas_identical": same, "train_steps": c["train_steps"],
               "episodes_rank0": c["episodes"]}, flush=True)
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
