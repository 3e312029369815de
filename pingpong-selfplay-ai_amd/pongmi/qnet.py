"""QNet parameter blocks and the K2 launches (pm_qnet_fold / pm_qnet_q / pm_qnet_act).

A QNet (models/qnet.py:52-75) lives on the device as one packed fp32 block of PM_QNET_NP floats in
state_dict order (features, then the 520 NoisyNet head parameters in the order Adam sees them,
then the epsilon buffers). Acting uses "effective" weights (NoisyLinear folded: mu, or
mu + sigma*eps) of PM_QNET_NW floats.
"""
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import PM_QNET_NP, PM_QNET_NW, check, ptr, stream_ptr

PARAM_LAYOUT = (
    ("features.0.weight", (64, 7)), ("features.0.bias", (64,)),
    ("features.2.weight", (64, 64)), ("features.2.bias", (64,)),
    ("fc_V.weight_mu", (1, 64)), ("fc_V.bias_mu", (1,)), ("fc_V.weight_sigma", (1, 64)), ("fc_V.bias_sigma", (1,)),
    ("fc_A.weight_mu", (3, 64)), ("fc_A.bias_mu", (3,)), ("fc_A.weight_sigma", (3, 64)), ("fc_A.bias_sigma", (3,)),
    ("fc_V.weight_epsilon", (1, 64)), ("fc_V.bias_epsilon", (1,)),
    ("fc_A.weight_epsilon", (3, 64)), ("fc_A.bias_epsilon", (3,)),
)
HEAD_KEYS = tuple(k for k, _ in PARAM_LAYOUT[4:12])
assert sum(int(np.prod(s)) for _, s in PARAM_LAYOUT) == PM_QNET_NP


def pack_state_dict(sd, device="cuda"):
    """QNet state_dict (reference key names) -> packed [PM_QNET_NP] fp32 device tensor."""
    missing = [k for k, _ in PARAM_LAYOUT if k not in sd]
    if missing:
        raise KeyError(f"QNet state_dict lacks {missing}")
    parts = []
    for k, shape in PARAM_LAYOUT:
        t = torch.as_tensor(sd[k]).detach().to(torch.float32)
        if tuple(t.shape) != shape:
            raise ValueError(f"{k}: shape {tuple(t.shape)} != {shape}")
        parts.append(t.reshape(-1).cpu())
    return torch.cat(parts).to(device)


def unpack_state_dict(block):
    """Packed block -> OrderedDict in QNet.state_dict() key order (CPU tensors, cloned)."""
    flat = block.detach().to("cpu", torch.float32).reshape(-1)
    out, o = OrderedDict(), 0
    sizes = {k: s for k, s in PARAM_LAYOUT}
    vals = {}
    for k, s in PARAM_LAYOUT:
        n = int(np.prod(s))
        vals[k] = flat[o:o + n].reshape(s).clone()
        o += n
    for k in ("features.0.weight", "features.0.bias", "features.2.weight", "features.2.bias"):
        out[k] = vals[k]
    for h in ("fc_V", "fc_A"):  # NoisyLinear registration order: params then buffers
        for s in ("weight_mu", "bias_mu", "weight_sigma", "bias_sigma", "weight_epsilon", "bias_epsilon"):
            out[f"{h}.{s}"] = vals[f"{h}.{s}"]
    assert set(out) == set(sizes)
    return out


def fold(blocks, mode, seed=0, counter=0, counter_dev=None, params_out=None, stream=None):
    """Effective weights [k, PM_QNET_NW] for k packed blocks ([k, NP] or [NP])."""
    lib = _lib.load()
    b = blocks.reshape(-1, PM_QNET_NP)
    _lib.require_device(b, "params")
    w = torch.zeros((b.shape[0], PM_QNET_NW), dtype=torch.float32, device=b.device)  # pads stay 0 (deterministic images)
    check(lib.pm_qnet_fold(ptr(b), ptr(params_out), int(mode), int(seed), int(counter), ptr(counter_dev), ptr(w),
                           b.shape[0], stream_ptr(stream)), "pm_qnet_fold")
    return w


def q_values(w_eff, x, stream=None):
    """QNet.forward on effective weights: x [n, 7] -> [n, 3] (one launch)."""
    lib = _lib.load()
    x = x.to(torch.float32).contiguous()
    _lib.require_device(x, "x")
    n = x.shape[0]
    q = torch.empty((n, 3), dtype=torch.float32, device=x.device)
    check(lib.pm_qnet_q(ptr(w_eff.contiguous()), ptr(x), ptr(q), n, stream_ptr(stream)), "pm_qnet_q")
    return q


def act(w_opp, opp_id, w_B, obsA, obsB, epsilon=0.0, seed=0, counter=0, eps_dev=None, counter_dev=None,
        want_q=False, chunk0=0, chunk1=0, stream=None):
    """Both players' actions (fused K2): aA = argmax Q_opp(obsA), aB = eps-greedy argmax Q_B(obsB)."""
    lib = _lib.load()
    n = obsA.shape[0]
    dev = obsA.device
    w_opp = w_opp.reshape(-1, PM_QNET_NW).contiguous()
    aA = torch.empty(n, dtype=torch.int8, device=dev)
    aB = torch.empty(n, dtype=torch.int8, device=dev)
    qA = torch.empty((n, 3), dtype=torch.float32, device=dev) if want_q else None
    qB = torch.empty((n, 3), dtype=torch.float32, device=dev) if want_q else None
    if opp_id is not None:
        opp_id = opp_id.to(device=dev, dtype=torch.int32).contiguous()
    check(lib.pm_qnet_act(ptr(w_opp), ptr(opp_id), w_opp.shape[0], ptr(w_B.contiguous()), ptr(obsA.contiguous()),
                          ptr(obsB.contiguous()), float(epsilon), ptr(eps_dev), int(seed), int(counter),
                          ptr(counter_dev), ptr(aA), ptr(aB), ptr(qA), ptr(qB), n, int(chunk0), int(chunk1),
                          stream_ptr(stream)), "pm_qnet_act")
    return (aA, aB, qA, qB) if want_q else (aA, aB)
