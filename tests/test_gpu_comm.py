"""The library-owned RCCL communicator (pm_comm_*, pongmi.dist.NativeComm) and the one-call sharded
vector steps (pm_selfplay_step_sharded, pm_rnn_selfplay_step_sharded) on ONE device: a 1-rank
nccl (RCCL) group, so the all-reduce is the identity and the sharded step must equal, bit for bit,
the unfused launch sequence the Python learner issues (k_actenv, k_learn, k_adam / DRQN grads +
apply). Multi-rank sums are RCCL's own; the gloo tests (test_distributed_cpu.py) cover the sharded
arithmetic with world 2.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from test_gpu_selfplay import _learner, _snap  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def comm():
    import torch.distributed as dist

    from pongmi.dist import NativeComm
    own = not dist.is_initialized()
    if own:
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    c = NativeComm()
    yield c
    c.close()
    if own:
        dist.destroy_process_group()


def test_allreduce_one_rank_is_identity(comm):
    x = torch.randn(10_000, device="cuda")
    y = x.clone()
    comm(y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    with pytest.raises(Exception):
        comm(torch.zeros(4, dtype=torch.float64, device="cuda"))


@pytest.mark.parametrize("U", [1, 3])
def test_sharded_step_equals_launch_sequence(golden, comm, U):
    kw = dict(n=1024, batch=256, cap=4096, seed=11, fuse_apply=False, updates_per_step=U)
    A = _learner(golden, **kw)                   # Python sequence: step_overlap / learn_ex + apply_ex
    B = _learner(golden, allreduce=comm, **kw)   # one library call per vector step
    for k in range(40):
        A.step()
        B.step()
        if k % 13 == 12:
            sa, sb = _snap(A), _snap(B)
            for key in sa:
                if key == "ctrl":
                    assert sa[key] == sb[key]
                else:
                    bad = np.argwhere(sa[key] != sb[key])
                    assert len(bad) == 0, (k, key, len(bad), bad[:4].tolist(), sa[key][tuple(bad[0])],
                                           sb[key][tuple(bad[0])])
    assert A.counters()["train_steps"] > 0


@pytest.mark.parametrize("clip", [1e6, 1e-3])
def test_rnn_sharded_step_equals_update(golden, comm, clip):
    from test_gpu_rnn_selfplay import _learner as rnn_learner
    # The sharded step (grads -> RCCL all-reduce -> apply, whose k_dq_norm forms the clip norm's shares
    # of the summed gradient) against pm_drqn_update (the shares from k_dq_wgrad's tiles): the same
    # order (round 6), so with one rank the parameters are bit-identical with the clip inactive (1e6)
    # and active on every update (1e-3).
    kw = dict(n=512, n_pool=1, epsilon=0.5, memory_size=2000, min_episodes_for_training_start=1, seed=4,
              grad_clip_norm=clip)
    A = rnn_learner(golden, **kw)
    B = rnn_learner(golden, allreduce=comm, **kw)
    for _ in range(50):
        A.step()
        B.step()
    torch.cuda.synchronize()
    assert torch.equal(A.learner.params, B.learner.params)
    assert torch.equal(A.trans, B.trans)
    assert A.counters() == B.counters()
    assert A.learner.stats()["steps"] == B.learner.stats()["steps"] > 0
