"""Sharding of the self-play learner over GPUs (one process per GPU, torch.distributed).

The path partitions by arena: every rank owns `n` arenas, its own replay ring and PER priorities,
and draws its serves / opponents / epsilon / PER uniforms from a rank-specific Philox key. The
only exchange is ONE sum all-reduce per update of the learner's gradient buffer (520 head
gradients, the finished-episode count and the "updated" flag — 2 112 bytes), after which every
rank applies the identical Adam step to identical parameters (grads divided by world inside the
apply kernel), so the replicas never diverge. NoisyNet noise uses a rank-independent key.
On ROCm the "nccl" backend is RCCL (xGMI between the GPUs of a node).
"""
import os

import torch

MASK64 = 0xFFFFFFFFFFFFFFFF


def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & MASK64
    return x ^ (x >> 31)


def shard_seeds(seed, rank):
    """(seed_env, seed_net): env-side draws differ per rank, network noise is shared."""
    seed_env = splitmix64((int(seed) * 0x100000001B3 + 1 + int(rank)) & MASK64)
    seed_net = splitmix64((int(seed) ^ 0x5EED5EED5EED) & MASK64)
    return seed_env, seed_net


def env_rank():
    """(rank, world, local_rank) from the torchrun environment (1 process = defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init(backend=None):
    """Initialise the default process group when WORLD_SIZE > 1; returns (rank, world, local_rank)."""
    rank, world, local = env_rank()
    if world > 1 and not torch.distributed.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        torch.distributed.init_process_group(backend, **kw)
    return rank, world, local


def grad_allreduce(group=None):
    """The learner's exchange step: in-place SUM all-reduce of the gradient buffer."""
    def allreduce(t):
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM, group=group)
    return allreduce


def max_over_ranks(value, device):
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(values, device):
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]
