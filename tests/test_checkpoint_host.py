"""Checkpoint formats (pongmi.checkpoint) on the host: the Adam state_dict the learners write loads
into a torch.optim.Adam over parameters of the same shapes and steps identically to one that made
those moments itself (train_iterative.py:101-104, train_rnn_iterative.py:641-652)."""
import torch

from pongmi import checkpoint

SHAPES = [(1, 64), (1,), (1, 64), (1,), (3, 64), (3,), (3, 64), (3,)]


def _adam_run(steps, seed=0):
    g = torch.Generator().manual_seed(seed)
    ps = [torch.randn(s, generator=g).requires_grad_() for s in SHAPES]
    opt = torch.optim.Adam(ps, lr=2.5e-4)
    for _ in range(steps):
        opt.zero_grad()
        sum((p * torch.randn(p.shape, generator=g)).sum() for p in ps).backward()
        opt.step()
    return ps, opt


def test_adam_state_dict_round_trip_and_load():
    ps, opt = _adam_run(3)
    sd = opt.state_dict()
    m, v, step = checkpoint.adam_moments(sd, SHAPES)
    assert step == 3 and m.numel() == sum(int(torch.tensor(s).prod()) for s in SHAPES)
    mine = checkpoint.adam_state_dict(SHAPES, m, v, step, lr=2.5e-4)
    assert mine["param_groups"] == sd["param_groups"]
    assert sorted(mine["state"]) == sorted(sd["state"])
    for i in sd["state"]:
        for k in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(torch.as_tensor(mine["state"][i][k]), torch.as_tensor(sd["state"][i][k])), (i, k)
    # the written dict drives a fresh optimizer to the same next step
    ps2 = [p.detach().clone().requires_grad_() for p in ps]
    opt2 = torch.optim.Adam(ps2, lr=2.5e-4)
    opt2.load_state_dict(mine)
    for a, b in ((ps, opt), (ps2, opt2)):
        b.zero_grad()
        sum(p.sum() for p in a).backward()
        b.step()
    for p, q in zip(ps, ps2):
        assert torch.equal(p, q)


def test_adam_state_dict_before_first_step_is_empty():
    sd = checkpoint.adam_state_dict(SHAPES, torch.zeros(520), torch.zeros(520), 0, lr=1e-4)
    assert sd["state"] == {} and sd["param_groups"][0]["params"] == list(range(8))
    ps = [torch.zeros(s, requires_grad=True) for s in SHAPES]
    torch.optim.Adam(ps, lr=1e-4).load_state_dict(sd)


def test_cpu_state_keeps_order_and_copies(tmp_path):
    sd = {"b": torch.ones(2), "a": torch.zeros(3, 2).t()}
    out = checkpoint.cpu_state(sd)
    assert list(out) == ["b", "a"]
    out["b"][0] = 5.0
    assert sd["b"][0] == 1.0  # a copy, not a view of the learner's buffers
    torch.save({"m": out}, tmp_path / "x.pth")
    back = checkpoint.load(tmp_path / "x.pth")
    assert torch.equal(back["m"]["a"], sd["a"])
