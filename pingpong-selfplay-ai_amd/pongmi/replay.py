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


class DeviceReplay:
    """The replay ring of PrioritizedReplay (train_iterative.py:49-63) as device buffers, filled by the
    collecting rollout (pongmi.rollout.SelfPlayRollout.run(..., replay=...), pm_rollout_push):
    trans [cap][PM_TRANS_F] rows (s[7], r, s'[7], bits(a | done << 8)), prios [cap], and the PER sum
    tree of pm_per_sample (`work`), which every collecting launch leaves current. pos / size mirror
    memory.pos / len(memory.buffer); max_prio is the priority the next push stores (max(prios), 1.0
    while empty, :57) — pushes never change it, so it is tracked here; call refresh() after
    changing prios by other means (it also rebuilds the sum tree)."""

    def __init__(self, cap, device, alpha=0.6):
        self.cap = int(cap)
        if self.cap <= 0:
            raise ValueError("cap must be > 0")
        self.alpha = float(alpha)
        self.trans = torch.zeros((self.cap, _lib.PM_TRANS_F), dtype=torch.float32, device=device)
        self.prios = torch.zeros(self.cap, dtype=torch.float32, device=device)
        nbytes = _lib.load().pm_per_work_bytes(self.cap)
        self.work = torch.zeros(max(nbytes, 256), dtype=torch.uint8, device=device)
        self.pos = 0
        self.size = 0
        self.max_prio = 1.0

    def push_prio(self):
        return self.max_prio if self.size > 0 else 1.0

    def advance(self, pushed):
        self.pos = (self.pos + pushed) % self.cap
        self.size = min(self.cap, self.size + pushed)

    def refresh(self):
        """After the host changed prios: rebuild the sum tree (pm_per_build) and the tracked max."""
        check(_lib.load().pm_per_build(ptr(self.prios), self.cap, self.alpha, ptr(self.work), stream_ptr()),
              "pm_per_build")
        self.max_prio = float(self.prios[:self.size].max()) if self.size else 1.0

    def leaves(self):
        """The PER leaves (prio^alpha, f32 [cap]) inside the tree workspace."""
        off = _pad(-(-self.cap // 1024)) + _pad(-(-self.cap // 64))
        return self.work[off:off + 4 * self.cap].view(torch.float32)

    def sample(self, bs, beta, seed=0, counter=0, uniforms=None):
        return per_sample(self.prios, self.size, bs, beta, alpha=self.alpha, uniforms=uniforms, seed=seed,
                          counter=counter)


def _pad(n_doubles):
    return ((n_doubles * 8 + 255) // 256) * 256
