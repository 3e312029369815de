"""The CPU baselines bench.py times (oracle/cpu_selfplay.py): the collecting rollout's port pushes
transitions with the training loop's layout (train_iterative.py:242-243): consecutive rows of an
arena chain s' -> s unless the episode ended, done rides in bits 8.. of float slot 15."""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def nets():
    from models.qnet import QNet
    import torch
    torch.manual_seed(0)
    sd = {k: v.numpy() for k, v in QNet(7, 3).state_dict().items()}
    return sd


def test_cpu_rollout_push_layout(nets):
    from oracle.cpu_selfplay import CpuRollout
    n, steps = 64, 40
    cpu = CpuRollout({}, n, nets, nets, epsilon=0.5, replay_cap=n * steps)
    for _ in range(steps):
        cpu.step()
    assert cpu.pos == 0
    assert np.all(cpu.prios == 1.0) and np.all(cpu.leaves == 1.0)
    rows = cpu.trans.reshape(steps, n, 16)
    bits = rows[..., 15].view(np.int32)
    act, done = bits & 0xFF, bits >> 8
    assert set(np.unique(act)) <= {0, 1, 2} and set(np.unique(done)) <= {0, 1}
    assert done.sum() > 0
    for k in range(1, steps):
        keep = done[k - 1] == 0
        assert np.array_equal(rows[k, keep, 0:7], rows[k - 1, keep, 8:15])
    assert set(np.unique(rows[..., 7])) <= {-1.0, 0.0, 1.0}
