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


def rccl_library_path():
    """The RCCL shared library the process runs: torch's bundled librccl.so (libtorch_hip loads it at
    `import torch`), else ROCm's."""
    for p in (os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so"), "/opt/rocm/lib/librccl.so.1"):
        if os.path.exists(p):
            return p
    raise FileNotFoundError("no librccl.so found (torch/lib, /opt/rocm/lib)")


class NativeComm:
    """The learner's gradient all-reduce as a libpongmi-owned RCCL communicator over the ranks of a
    torch.distributed group (pm_comm_*, include/pongmi.h). Passed as a learner's `allreduce`, it makes
    every sharded vector step ONE library call (pm_selfplay_step_sharded / pm_rnn_selfplay_step_sharded)
    with ncclAllReduce on the learner's stream; called on a tensor it is an in-place SUM all-reduce.

    Rank 0 creates the RCCL id and broadcasts it with a status byte over the group, so a failure to
    bind RCCL raises on every rank (no rank is left waiting in ncclCommInitRank)."""

    def __init__(self, group=None, rccl_path=None):
        import ctypes

        import torch.distributed as dist

        from . import _lib
        self._lib = lib = _lib.load()
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        path = (rccl_path or rccl_library_path()).encode()
        buf = torch.zeros(_lib.PM_COMM_ID_BYTES + 1, dtype=torch.uint8)
        err = ""
        if self.rank == 0:
            rc = lib.pm_comm_unique_id(path, buf.data_ptr())
            if rc == 0:
                buf[-1] = 1
            else:
                err = lib.pm_last_error().decode(errors="replace")
        on_dev = dist.get_backend(group) == "nccl"
        t = buf.cuda() if on_dev else buf
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        buf = t.cpu()
        if int(buf[-1]) != 1:
            raise _lib.PongmiError(f"pm_comm_unique_id failed on rank 0: {err or 'see rank 0'}")
        h = ctypes.c_void_p()
        _lib.check(lib.pm_comm_init(path, buf.data_ptr(), self.world, self.rank, ctypes.byref(h)), "pm_comm_init")
        self.handle = h

    def info(self):
        """(nranks, rank, device) as RCCL reports them for this communicator (pm_comm_info)."""
        import ctypes

        from . import _lib
        n, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._lib.pm_comm_info(self.handle, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)),
                   "pm_comm_info")
        return n.value, r.value, d.value

    @property
    def pm_comm(self):
        return self.handle

    def __call__(self, t):
        from . import _lib
        _lib.require_device(t, "all-reduce buffer")
        if t.dtype != torch.float32:
            raise _lib.PongmiError("NativeComm all-reduces float32 buffers")
        _lib.check(self._lib.pm_comm_allreduce_f32(self.handle, t.data_ptr(), t.numel(), _lib.stream_ptr()),
                   "pm_comm_allreduce_f32")

    def close(self):
        if self.handle:
            from . import _lib
            h, self.handle = self.handle, None
            _lib.check(self._lib.pm_comm_destroy(h), "pm_comm_destroy")
