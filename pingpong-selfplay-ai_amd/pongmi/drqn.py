"""The DRQN learner (K6): train_step_rnn (scripts/train_rnn_iterative.py:400-531) on device buffers.

DRQNLearner owns modelB's and targetB's packed QNetRNN blocks (pongmi.rnn layout), the Adam moments
and the update workspace; update() runs one train_step_rnn on a sampled batch of sequences
(obs / next [B, T, 7], act / rew / done [B, T]) as one pm_drqn_update call: forward of modelB on obs
and next and targetB on next from zero state, double-DQN target, smooth-L1, BPTT, clip_grad_norm_,
Adam, target sync every target_update_interval steps — no host synchronisation.

For data-parallel training, grads() / apply() split the update around the gradient all-reduce:
every rank computes its gradient into `grad` ([PM_RNN_NPARAM] gradients, then a 1 marking a
contributing rank), the ranks sum `grad` (one all-reduce), then apply() divides by the number of
contributing ranks and runs the clip on the global norm and the identical Adam step on every rank.
A rank whose `enable` flag is 0 (its sequence buffer not yet full enough) contributes zeros.
"""
import ctypes

import torch

from . import _lib
from ._lib import PM_RNN_NP, PM_RNN_NPARAM, check, stream_ptr
from .checkpoint import adam_moments, adam_state_dict
from .rnn import PARAM_LAYOUT, PARAM_KEYS, pack_state_dict, unpack_state_dict

PARAM_SHAPES = [s for k, s in PARAM_LAYOUT if k in PARAM_KEYS]  # modelB.parameters() order


class DRQNLearner:
    def __init__(self, modelB, target=None, *, batch=64, T=8, gamma=0.99, lr=1e-4, betas=(0.9, 0.999), eps=1e-8,
                 max_norm=1.0, target_update_interval=2000, enable=None, device="cuda", poll_limit=0):
        """modelB / target: a QNetRNN module, its state_dict, or a packed [PM_RNN_NP] tensor;
        target None = a copy of modelB (targetB.load_state_dict(modelB.state_dict()), :336-338)."""
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.params = self._block(modelB)
        self.target = self._block(target) if target is not None else self.params.clone()
        self.adam_m = torch.zeros(PM_RNN_NPARAM, dtype=torch.float32, device=self.device)
        self.adam_v = torch.zeros(PM_RNN_NPARAM, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(PM_RNN_NPARAM + 4, dtype=torch.float32, device=self.device)
        self.batch, self.T = int(batch), int(T)
        nbytes = self.lib.pm_drqn_work_bytes(self.batch, self.T)
        if nbytes < 0:
            raise ValueError("invalid batch / T")
        # zero-filled before first use (pm_drqn_init below): the hand-off slots' tags and the tag epoch
        # (flags[0]) must not start as whatever the allocator hands back
        self.work = torch.empty((nbytes + 15) // 16 * 4, dtype=torch.float32, device=self.device)
        self.stats_buf = torch.zeros(ctypes.sizeof(_lib.DrqnStats), dtype=torch.uint8, device=self.device)
        self.obs = torch.zeros((self.batch, self.T, 7), dtype=torch.float32, device=self.device)
        self.next = torch.zeros_like(self.obs)
        self.act = torch.zeros((self.batch, self.T), dtype=torch.int32, device=self.device)
        self.rew = torch.zeros((self.batch, self.T), dtype=torch.float32, device=self.device)
        self.done = torch.zeros((self.batch, self.T), dtype=torch.uint8, device=self.device)
        d = _lib.Drqn()
        for name in ("params", "target", "adam_m", "adam_v", "grad", "work", "obs", "next", "act", "rew", "done"):
            setattr(d, name, getattr(self, name).data_ptr())
        d.stats = self.stats_buf.data_ptr()
        self.enable = enable  # optional int32 device flag (the self-play sampler's)
        d.enable = enable.data_ptr() if enable is not None else None
        d.batch, d.T = self.batch, self.T
        d.target_update_interval = int(target_update_interval)
        d.gamma, d.lr, d.beta1, d.beta2, d.adam_eps, d.max_norm = float(gamma), float(lr), float(betas[0]), \
            float(betas[1]), float(eps), float(max_norm)
        d.poll_limit = int(poll_limit)  # 0: the library default; < 0 is the tests' forced-timeout hook
        self.desc = d
        self._call(self.lib.pm_drqn_init)  # the workspace zero-filled by the library (pongmi.h, ABI 20)

    def _block(self, m):
        if isinstance(m, torch.Tensor):
            if m.numel() != PM_RNN_NP:
                raise ValueError(f"packed QNetRNN block must have {PM_RNN_NP} floats")
            return m.detach().to(self.device, torch.float32).reshape(-1).clone()
        sd = m.state_dict() if hasattr(m, "state_dict") else m
        return pack_state_dict(sd, self.device)

    def load_batch(self, obs, act, rew, next_obs, done):
        """Copy a sampled batch (any device / dtype) into the learner's input buffers."""
        self.obs.copy_(torch.as_tensor(obs).reshape(self.obs.shape))
        self.next.copy_(torch.as_tensor(next_obs).reshape(self.next.shape))
        self.act.copy_(torch.as_tensor(act).reshape(self.act.shape))
        self.rew.copy_(torch.as_tensor(rew).reshape(self.rew.shape))
        self.done.copy_(torch.as_tensor(done).reshape(self.done.shape))

    def _call(self, fn, stream=None):
        check(fn(ctypes.byref(self.desc), stream_ptr(stream)), fn.__name__)

    def update(self, *batch, stream=None):
        """One train_step_rnn; batch = (obs, act, rew, next_obs, done) or nothing (buffers already filled)."""
        if batch:
            self.load_batch(*batch)
        self._call(self.lib.pm_drqn_update, stream)

    def grads(self, *batch, stream=None):
        if batch:
            self.load_batch(*batch)
        self._call(self.lib.pm_drqn_grads, stream)

    def apply(self, stream=None):
        self._call(self.lib.pm_drqn_apply, stream)

    def stats(self):
        """(steps, loss, pre-clip grad norm, mean q, status) of the last update (host sync). status
        (latched) 2: a hand-off inside pm_drqn_grads timed out on this replica; 4: (before round 6) the
        apply's norm arrival timed out; 8: an update was voided (a timeout on any rank: parameters, Adam
        state, step count and target left as they were)."""
        s = _lib.DrqnStats.from_buffer_copy(bytes(self.stats_buf.cpu().numpy()))
        return dict(steps=s.steps, adam_t=s.adam_t, loss=s.loss, norm=s.norm, q_mean=s.q_mean, status=s.status)

    def check_status(self):
        """Raise when any update was voided or partly applied (status bits above; host sync)."""
        st = self.stats()["status"]
        if st & 14:
            raise _lib.PongmiError(f"DRQN update: device status {st} (2: hand-off timed out, 4: apply arrival "
                                   f"timed out, 8: update voided)")
        return st

    def state_dict(self):
        """modelB's state_dict (reference key names)."""
        return unpack_state_dict(self.params)

    # ------------------------------------------------------------------ optimizer / counters
    def _stats(self):
        return _lib.DrqnStats.from_buffer_copy(bytes(self.stats_buf.cpu().numpy()))

    def _set_stats(self, **kw):
        s = self._stats()
        for k, v in kw.items():
            setattr(s, k, v)
        self.stats_buf.copy_(torch.frombuffer(bytearray(bytes(s)), dtype=torch.uint8))

    def optimizer_state_dict(self):
        """torch.optim.Adam(modelB.parameters(), lr).state_dict() equivalent (train_rnn_iterative.py:335)."""
        return adam_state_dict(PARAM_SHAPES, self.adam_m, self.adam_v, self._stats().adam_t, self.desc.lr,
                               (self.desc.beta1, self.desc.beta2), self.desc.adam_eps)

    def load_optimizer_state_dict(self, sd):
        m, v, step = adam_moments(sd, PARAM_SHAPES)
        self.adam_m.copy_(m)
        self.adam_v.copy_(v)
        self._set_stats(adam_t=step)

    def new_optimizer(self):
        """optimizerB = optim.Adam(modelB.parameters(), lr=lr): zero moments, step 0."""
        self.adam_m.zero_()
        self.adam_v.zero_()
        self._set_stats(adam_t=0)

    def set_train_steps(self, steps):
        self._set_stats(steps=int(steps))

    def load_params(self, modelB, target=None):
        """modelB <- state; targetB <- target (default: a copy of the new modelB)."""
        self.params.copy_(self._block(modelB))
        self.target.copy_(self._block(target) if target is not None else self.params)

    def target_state_dict(self):
        return unpack_state_dict(self.target)
