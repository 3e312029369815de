"""QNetRNN parameter blocks and the K5 launches (pm_rnn_fold / pm_rnn_q / pm_rnn_act).

A QNetRNN (models/qnet_rnn.py:53-152, the default 7 -> 64 -> 128 -> LSTM 128 -> 128 -> V/A shape)
lives on the device as one packed fp32 block of PM_RNN_NP floats: its parameters in
modelB.parameters() order (the order Adam sees them, train_rnn_iterative.py:323), then the three
NoisyLinear layers' epsilon buffers. Acting uses effective weights (NoisyLinear folded, the LSTM
biases summed) of PM_RNN_NW floats in MFMA fragment order.

The recurrent state (h, c) of n arenas is two [n, 128] fp32 device arrays, advanced in place.
"""
from collections import OrderedDict

import numpy as np
import torch

from . import _lib
from ._lib import PM_RNN_NP, PM_RNN_NPARAM, PM_RNN_NW, check, ptr, stream_ptr

HIDDEN = 128


def _noisy(name, n_in, n_out):
    return ((f"{name}.weight_mu", (n_out, n_in)), (f"{name}.bias_mu", (n_out,)),
            (f"{name}.weight_sigma", (n_out, n_in)), (f"{name}.bias_sigma", (n_out,)))


PARAM_LAYOUT = (
    ("features_extractor.0.weight", (64, 7)), ("features_extractor.0.bias", (64,)),
    ("features_extractor.2.weight", (128, 64)), ("features_extractor.2.bias", (128,)),
    ("lstm.weight_ih_l0", (512, 128)), ("lstm.weight_hh_l0", (512, 128)),
    ("lstm.bias_ih_l0", (512,)), ("lstm.bias_hh_l0", (512,)),
) + _noisy("fc_shared_head.0", 128, 128) + _noisy("fc_V", 128, 1) + _noisy("fc_A", 128, 3) + (
    ("fc_shared_head.0.weight_epsilon", (128, 128)), ("fc_shared_head.0.bias_epsilon", (128,)),
    ("fc_V.weight_epsilon", (1, 128)), ("fc_V.bias_epsilon", (1,)),
    ("fc_A.weight_epsilon", (3, 128)), ("fc_A.bias_epsilon", (3,)),
)
PARAM_KEYS = tuple(k for k, _ in PARAM_LAYOUT if "epsilon" not in k)  # modelB.parameters() order
assert sum(int(np.prod(s)) for _, s in PARAM_LAYOUT) == PM_RNN_NP
assert sum(int(np.prod(s)) for k, s in PARAM_LAYOUT if k in PARAM_KEYS) == PM_RNN_NPARAM

# QNetRNN.state_dict() key order (modules in registration order; NoisyLinear params then buffers)
STATE_KEYS = tuple(k for k, _ in PARAM_LAYOUT[:8]) + tuple(
    f"{m}.{s}" for m in ("fc_shared_head.0", "fc_V", "fc_A")
    for s in ("weight_mu", "bias_mu", "weight_sigma", "bias_sigma", "weight_epsilon", "bias_epsilon"))


def pack_state_dict(sd, device="cuda"):
    """QNetRNN state_dict (reference key names) -> packed [PM_RNN_NP] fp32 device tensor."""
    missing = [k for k, _ in PARAM_LAYOUT if k not in sd]
    if missing:
        raise KeyError(f"QNetRNN state_dict lacks {missing}")
    parts = []
    for k, shape in PARAM_LAYOUT:
        t = torch.as_tensor(sd[k]).detach().to(torch.float32)
        if tuple(t.shape) != shape:
            raise ValueError(f"{k}: shape {tuple(t.shape)} != {shape} (only the default QNetRNN shape is packed)")
        parts.append(t.reshape(-1).cpu())
    return torch.cat(parts).to(device)


def unpack_state_dict(block):
    """Packed block -> OrderedDict in QNetRNN.state_dict() key order (CPU tensors, cloned)."""
    flat = block.detach().to("cpu", torch.float32).reshape(-1)
    vals, o = {}, 0
    for k, s in PARAM_LAYOUT:
        n = int(np.prod(s))
        vals[k] = flat[o:o + n].reshape(s).clone()
        o += n
    return OrderedDict((k, vals[k]) for k in STATE_KEYS)


def fold(blocks, mode, seed=0, counter=0, counter_dev=None, params_out=None, stream=None):
    """Effective weights [k, PM_RNN_NW] for k packed blocks ([k, NP] or [NP])."""
    lib = _lib.load()
    b = blocks.reshape(-1, PM_RNN_NP).contiguous()
    _lib.require_device(b, "params")
    w = torch.zeros((b.shape[0], PM_RNN_NW), dtype=torch.float32, device=b.device)  # pads stay 0 (deterministic images)
    check(lib.pm_rnn_fold(ptr(b), ptr(params_out), int(mode), int(seed), int(counter), ptr(counter_dev), ptr(w),
                          b.shape[0], stream_ptr(stream)), "pm_rnn_fold")
    return w


def init_state(n, device="cuda"):
    """Zero (h, c), each [n, 128] (QNetRNN.init_hidden, models/qnet_rnn.py:146-152, without the layer axis)."""
    return (torch.zeros((n, HIDDEN), dtype=torch.float32, device=device),
            torch.zeros((n, HIDDEN), dtype=torch.float32, device=device))


def _state(t, n, name):
    if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (n, HIDDEN):
        raise ValueError(f"{name} must be a contiguous float32 [{n}, {HIDDEN}] tensor")
    _lib.require_device(t, name)
    return t


def q_step(w_eff, x, h, c, reset=None, stream=None):
    """One QNetRNN step (T = 1) on effective weights: x [n, 7]; (h, c) [n, 128] advanced in place;
    reset [n] bool/uint8 (optional) starts those rows from zero state. Returns q [n, 3]."""
    lib = _lib.load()
    x = x.to(torch.float32).contiguous()
    _lib.require_device(x, "x")
    n = x.shape[0]
    _state(h, n, "h")
    _state(c, n, "c")
    if reset is not None:
        reset = reset.to(device=x.device, dtype=torch.uint8).contiguous()
    q = torch.empty((n, 3), dtype=torch.float32, device=x.device)
    check(lib.pm_rnn_q(ptr(w_eff.contiguous()), ptr(x), ptr(h), ptr(c), ptr(reset), ptr(q), n, stream_ptr(stream)),
          "pm_rnn_q")
    return q


def forward(w_eff, x_seq, h0=None, c0=None, stream=None):
    """QNetRNN.forward (models/qnet_rnn.py:107-144): x_seq [B, T, 7] from (h0, c0) [B, 128]
    (None: zeros) -> (q of the last step [B, 3], h_n [B, 128], c_n [B, 128]); T launches."""
    B, T, _ = x_seq.shape
    if T < 1:
        raise ValueError("sequence length must be >= 1")
    dev = x_seq.device
    h = torch.zeros((B, HIDDEN), dtype=torch.float32, device=dev) if h0 is None else \
        h0.to(device=dev, dtype=torch.float32).reshape(B, HIDDEN).clone()
    c = torch.zeros((B, HIDDEN), dtype=torch.float32, device=dev) if c0 is None else \
        c0.to(device=dev, dtype=torch.float32).reshape(B, HIDDEN).clone()
    x_seq = x_seq.to(torch.float32)
    q = None
    for t in range(T):
        q = q_step(w_eff, x_seq[:, t], h, c, stream=stream)
    return q, h, c


def act(w_opp, opp_id, w_B, obsA, obsB, stA, stB, reset=None, epsilon=0.0, seed=0, counter=0, eps_dev=None,
        counter_dev=None, want_q=False, chunk0=0, chunk1=0, opp_list=None, opp_cnt=None, stream=None):
    """Both players' QNetRNN actions (fused K5): aA = argmax Q_opp(obsA; stA) greedy,
    aB = eps-greedy argmax Q_B(obsB; stB); stA = (hA, cA), stB = (hB, cB) advance in place."""
    lib = _lib.load()
    n = obsA.shape[0]
    dev = obsA.device
    w_opp = w_opp.reshape(-1, PM_RNN_NW).contiguous()
    hA, cA = (_state(t, n, nm) for t, nm in zip(stA, ("hA", "cA")))
    hB, cB = (_state(t, n, nm) for t, nm in zip(stB, ("hB", "cB")))
    aA = torch.empty(n, dtype=torch.int8, device=dev)
    aB = torch.empty(n, dtype=torch.int8, device=dev)
    qA = torch.empty((n, 3), dtype=torch.float32, device=dev) if want_q else None
    qB = torch.empty((n, 3), dtype=torch.float32, device=dev) if want_q else None
    if opp_id is not None:
        opp_id = opp_id.to(device=dev, dtype=torch.int32).contiguous()
    if reset is not None:
        reset = reset.to(device=dev, dtype=torch.uint8).contiguous()
    check(lib.pm_rnn_act(ptr(w_opp), ptr(opp_id), w_opp.shape[0], ptr(w_B.contiguous()), ptr(obsA.contiguous()),
                         ptr(obsB.contiguous()), ptr(hA), ptr(cA), ptr(hB), ptr(cB), ptr(reset), float(epsilon),
                         ptr(eps_dev), int(seed), int(counter), ptr(counter_dev), ptr(aA), ptr(aB), ptr(qA), ptr(qB),
                         n, int(chunk0), int(chunk1), ptr(opp_list), ptr(opp_cnt), stream_ptr(stream)), "pm_rnn_act")
    return (aA, aB, qA, qB) if want_q else (aA, aB)
