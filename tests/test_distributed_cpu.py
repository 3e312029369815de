"""The sharded learner's exchange step on CPU: world_size 2 over gloo (the GPU path uses RCCL).

Each rank owns its arenas and replay, so its update batch (and gradient) differs; one SUM
all-reduce of the packed buffer [520 head grads | finished episodes | updated flag] followed by
grads / world makes every rank apply the identical Adam step and the identical epsilon decay,
i.e. the replicas stay bit-identical and equal a single learner on the mean gradient."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle import oracle as orc
    from pongmi import dist as pd

    r, w, _ = pd.init(backend="gloo")
    assert (r, w) == (rank, world)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dqn_steps.npz")))
    sd = {k[5:]: v for k, v in g.items() if k.startswith("init.")}
    heads = orc.pack_heads(sd)
    m = np.zeros_like(heads)
    v = np.zeros_like(heads)
    eps_greedy = 1.0
    allreduce = pd.grad_allreduce()
    for step in range(3):
        k = f"s{step}."
        eps = {kk[len(k) + 7:]: vv for kk, vv in g.items() if kk.startswith(k + "noiseB.")}
        sl = slice(rank * 128, rank * 128 + 128)  # this rank's half of the batch = its own replay sample
        res = orc.dqn_loss_grads(sd, heads, heads, eps, g[k + "s"][sl], g[k + "a"][sl], g[k + "r"][sl],
                                 g[k + "ns"][sl], g[k + "d"][sl], g[k + "iw"][sl], 0.99)
        buf = torch.zeros(528, dtype=torch.float64)
        buf[:520] = torch.from_numpy(res["grads"])
        buf[520] = 10 + 7 * rank  # finished episodes on this shard
        buf[521] = 1.0
        allreduce(buf)
        gsum = buf[:520].numpy()
        heads, m, v = orc.adam_step(heads, gsum / world, m, v, step + 1, 2.5e-4)
        eps_greedy = max(0.02, eps_greedy * 0.995 ** float(buf[520]))
        assert float(buf[521]) == world
    seed_env, seed_net = pd.shard_seeds(7, rank)
    t = pd.max_over_ranks(1.0 + rank, "cpu")
    out_q.put((rank, heads, eps_greedy, seed_env, seed_net, t))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gradient_allreduce_keeps_replicas_identical():
    from oracle import oracle as orc
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, heads, eps, se, sn, t = q.get(timeout=100)
        res[r] = (heads, eps, se, sn, t)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    h0, e0, se0, sn0, t0 = res[0]
    h1, e1, se1, sn1, t1 = res[1]
    assert np.array_equal(h0, h1) and e0 == e1  # replicas identical
    assert se0 != se1 and sn0 == sn1  # env draws per shard, network noise shared
    assert t0 == t1 == 2.0  # max over ranks
    assert e0 == max(0.02, 0.995 ** (3 * 27))
    # equals one learner applying the mean of the two shards' gradients
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dqn_steps.npz")))
    sd = {k[5:]: v for k, v in g.items() if k.startswith("init.")}
    heads = orc.pack_heads(sd)
    m = np.zeros_like(heads)
    v = np.zeros_like(heads)
    for step in range(3):
        k = f"s{step}."
        eps = {kk[len(k) + 7:]: vv for kk, vv in g.items() if kk.startswith(k + "noiseB.")}
        gs = []
        for rank in range(world):
            sl = slice(rank * 128, rank * 128 + 128)
            gs.append(orc.dqn_loss_grads(sd, heads, heads, eps, g[k + "s"][sl], g[k + "a"][sl], g[k + "r"][sl],
                                         g[k + "ns"][sl], g[k + "d"][sl], g[k + "iw"][sl], 0.99)["grads"])
        heads, m, v = orc.adam_step(heads, (gs[0] + gs[1]) / world, m, v, step + 1, 2.5e-4)
    np.testing.assert_allclose(h0, heads, rtol=1e-12, atol=1e-15)


class _OracleShard:
    """One rank's learner with the launch methods pongmi.selfplay.sharded_vector_step calls, each
    backed by the oracle on the CPU (no device): learn_ex fills the PRODUCT's packed exchange buffer
    (layout from include/pongmi.h PM_GRAD_*, float32 as on the device) with the oracle's double-DQN
    gradients of this shard's half of the golden batch; apply_ex applies Adam to grads / world and the
    epsilon decay by the summed episode count, as k_adam does. `calls` records the launch sequence."""

    def __init__(self, orc, g, rank, world, overlap):
        from pongmi import _lib
        self.orc, self.g, self.rank, self.world, self.overlap = orc, g, rank, world, overlap
        self.sd = {k[5:]: v for k, v in g.items() if k.startswith("init.")}
        self.heads = orc.pack_heads(self.sd)
        self.m, self.v = np.zeros_like(self.heads), np.zeros_like(self.heads)
        self.eps, self.ts, self.upd = 1.0, 0, 0
        self.grad = torch.zeros(_lib.PM_GRAD_LEN, dtype=torch.float32)
        self._aA_ready = False
        self.calls, self.seen = [], []

    def act(self, part):
        self.calls.append("act_A")
        self._aA_ready = True

    def actenv(self):
        self.calls.append("actenv")
        self._aA_ready = False

    def rollout(self):
        self.calls.append("rollout")

    def resample(self):
        self.calls.append("resample")

    def learn_ex(self, mode, act_next=False):
        from pongmi import _lib
        self.calls.append(("learn", mode, bool(act_next)))
        k = f"s{self.upd % 3}."
        g = self.g
        eps = {kk[len(k) + 7:]: vv for kk, vv in g.items() if kk.startswith(k + "noiseB.")}
        sl = slice(self.rank * 128, self.rank * 128 + 128)  # this rank's own replay sample
        res = self.orc.dqn_loss_grads(self.sd, self.heads, self.heads, eps, g[k + "s"][sl], g[k + "a"][sl],
                                      g[k + "r"][sl], g[k + "ns"][sl], g[k + "d"][sl], g[k + "iw"][sl], 0.99)
        self.grad.zero_()
        self.grad[:_lib.PM_QNET_NHEAD] = torch.from_numpy(res["grads"].astype(np.float32))
        self.grad[_lib.PM_GRAD_EPISODES] = (10 + 7 * self.rank) if mode & _lib.PM_UPD_FIRST else 0
        self.grad[_lib.PM_GRAD_UPDATED] = 1.0
        if act_next:
            self._aA_ready = True

    def apply_ex(self, mode):
        from pongmi import _lib
        self.calls.append(("apply", mode))
        buf = self.grad.numpy().astype(np.float64)
        self.seen.append((buf[_lib.PM_GRAD_EPISODES], buf[_lib.PM_GRAD_UPDATED]))
        self.ts += 1
        self.upd += 1
        self.heads, self.m, self.v = self.orc.adam_step(self.heads, buf[:_lib.PM_QNET_NHEAD] / self.world, self.m,
                                                        self.v, self.ts, 2.5e-4)
        self.eps = max(0.02, self.eps * 0.995 ** buf[_lib.PM_GRAD_EPISODES])

    def commit(self):
        self.calls.append("commit")


def _product_worker(rank, world, port, out_q, U, overlap):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from oracle import oracle as orc
    from pongmi import dist as pd
    from pongmi.selfplay import sharded_vector_step

    pd.init(backend="gloo")
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dqn_steps.npz")))
    L = _OracleShard(orc, g, rank, world, overlap)
    for _ in range(2):
        sharded_vector_step(L, pd.grad_allreduce(), U)
    out_q.put((rank, L.heads, L.eps, L.calls, L.seen))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("U,overlap", [(1, True), (3, False)])
def test_product_sharded_step_sequence_over_gloo(U, overlap):
    """pongmi.selfplay.sharded_vector_step — the sequence SelfPlayLearner.step runs for world > 1 and
    the twin of pm_selfplay_step_sharded — over two gloo ranks: the launch order (act A once, actenv /
    rollout, per update resample + learn_ex + all-reduce + apply_ex, commit), the packed buffer after
    the SUM (episodes summed over the shards on update 0 only, the updated flag = world on every
    update), and replicas that stay bit-identical and equal one learner on the mean gradient."""
    from oracle import oracle as orc
    from pongmi import _lib
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_product_worker, args=(r, world, port, q, U, overlap)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, heads, eps, calls, seen = q.get(timeout=100)
        res[r] = (heads, eps, calls, seen)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    F, L_ = _lib.PM_UPD_FIRST, _lib.PM_UPD_LAST
    first = F | (L_ if U == 1 else 0)
    step = (["actenv"] if overlap else ["rollout"]) + [("learn", first, overlap), ("apply", first)]
    for u in range(1, U):
        step += ["resample", ("learn", 0, False), ("apply", 0)]
    step += ["commit"] if U > 1 else []
    expect = (["act_A"] if overlap else []) + step + step  # the next act rides the learner launch
    assert res[0][2] == expect and res[1][2] == expect
    for u, (ep, upd) in enumerate(res[0][3]):
        assert upd == world and ep == (10 + 17 if u % U == 0 else 0)
    assert np.array_equal(res[0][0], res[1][0]) and res[0][1] == res[1][1]  # replicas identical
    assert res[0][1] == max(0.02, 0.995 ** 27 * 0.995 ** 27)
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "dqn_steps.npz")))
    sd = {k[5:]: v for k, v in g.items() if k.startswith("init.")}
    heads = orc.pack_heads(sd)
    m, v = np.zeros_like(heads), np.zeros_like(heads)
    for t in range(2 * U):
        k = f"s{t % 3}."
        eps = {kk[len(k) + 7:]: vv for kk, vv in g.items() if kk.startswith(k + "noiseB.")}
        gs = [orc.dqn_loss_grads(sd, heads, heads, eps, g[k + "s"][sl], g[k + "a"][sl], g[k + "r"][sl],
                                 g[k + "ns"][sl], g[k + "d"][sl], g[k + "iw"][sl], 0.99)["grads"].astype(np.float32)
              for sl in (slice(0, 128), slice(128, 256))]
        heads, m, v = orc.adam_step(heads, (gs[0] + gs[1]).astype(np.float64) / world, m, v, t + 1, 2.5e-4)
    np.testing.assert_allclose(res[0][0], heads, rtol=1e-12, atol=1e-15)
