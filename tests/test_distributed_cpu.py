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
