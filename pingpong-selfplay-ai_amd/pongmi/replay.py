"""Prioritized replay on the device (K4: pm_per_sample / pm_per_update).

Mirrors PrioritizedReplay (scripts/train_iterative.py:49-76): proportional sampling of
prios[0:size]^alpha with replacement, IS weights (size * P(i))^-beta / max, priority update
|err| + 1e-6 with the last duplicate winning.
"""
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

_work = {}


def _workspace(cap, device):
    key = (int(cap), str(device))
    if key not in _work:
        nbytes = _lib.load().pm_per_work_bytes(int(cap))
        _work[key] = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
    return _work[key]


def per_sample(prios, size, bs, beta, alpha=0.6, uniforms=None, seed=0, counter=0, stream=None):
    """Returns (idx int64 [bs], weights f32 [bs]). `uniforms` (float64 [bs]) replays
    np.random.choice's own draws; None draws them from Philox(seed, counter)."""
    lib = _lib.load()
    _lib.require_device(prios, "prios")
    dev = prios.device
    idx = torch.empty(bs, dtype=torch.int64, device=dev)
    w = torch.empty(bs, dtype=torch.float32, device=dev)
    if uniforms is not None:
        uniforms = torch.as_tensor(uniforms, dtype=torch.float64).to(dev).contiguous()
    work = _workspace(prios.numel(), dev)
    check(lib.pm_per_sample(ptr(prios), int(size), float(alpha), float(beta), ptr(uniforms), int(seed), int(counter),
                            ptr(idx), ptr(w), int(bs), ptr(work), stream_ptr(stream)), "pm_per_sample")
    return idx, w


def per_update(prios, idx, errors, stream=None):
    lib = _lib.load()
    idx = idx.to(device=prios.device, dtype=torch.int64).contiguous()
    errors = errors.to(device=prios.device, dtype=torch.float32).contiguous()
    check(lib.pm_per_update(ptr(prios), ptr(idx), ptr(errors), idx.numel(), stream_ptr(stream)), "pm_per_update")
