"""Checkpoint I/O in the reference's formats.

The training scripts save plain dicts with torch.save (scripts/train_iterative.py:272-278,
scripts/train_rnn_iterative.py:641-652, :828-837, :863-872) whose tensors are module state_dicts
and a torch.optim.Adam state_dict. The learners keep parameters and Adam moments as flat device
buffers; these helpers convert both ways, and load checkpoints with weights_only=True.
"""
from collections import OrderedDict

import numpy as np
import torch


def load(path):
    """A checkpoint dict (torch.load, weights_only=True: tensors and plain containers only)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def adam_state_dict(shapes, m, v, step, lr, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.Adam.state_dict() for parameters of `shapes` with flat moments m, v (any device)
    after `step` steps. The param_group keys come from a real torch.optim.Adam of this torch build,
    so the dict loads into an optimizer over the same parameters."""
    proto = [torch.zeros(1, requires_grad=True) for _ in shapes]
    tmpl = torch.optim.Adam(proto, lr=lr, betas=betas, eps=eps).state_dict()
    m = m.detach().to("cpu", torch.float32).reshape(-1)
    v = v.detach().to("cpu", torch.float32).reshape(-1)
    state, o = {}, 0
    for i, s in enumerate(shapes):
        k = int(np.prod(s))
        if step > 0:  # torch creates per-parameter state on the first step
            state[i] = {"step": torch.tensor(float(step)), "exp_avg": m[o:o + k].reshape(s).clone(),
                        "exp_avg_sq": v[o:o + k].reshape(s).clone()}
        o += k
    return {"state": state, "param_groups": tmpl["param_groups"]}


def adam_moments(opt_sd, shapes):
    """(m, v, step) flat CPU tensors from an Adam state_dict over parameters of `shapes`."""
    n = sum(int(np.prod(s)) for s in shapes)
    m, v, step = torch.zeros(n), torch.zeros(n), 0
    o = 0
    for i, s in enumerate(shapes):
        k = int(np.prod(s))
        st = opt_sd.get("state", {}).get(i)
        if st:
            m[o:o + k] = torch.as_tensor(st["exp_avg"]).reshape(-1).float()
            v[o:o + k] = torch.as_tensor(st["exp_avg_sq"]).reshape(-1).float()
            step = int(float(st["step"]))
        o += k
    return m, v, step


def cpu_state(sd):
    """A state dict with contiguous CPU tensors (what the reference's checkpoints hold after load)."""
    return OrderedDict((k, torch.as_tensor(v).detach().to("cpu").clone()) for k, v in sd.items())
