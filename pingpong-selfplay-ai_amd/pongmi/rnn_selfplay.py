"""The batched QNetRNN self-play learner: scripts/train_rnn_iterative.py's hot loop (:731-798) for n
arenas per device — fold + act (K5) + env / sequence store (K7) + DRQN update (K6) per vector step
on one stream, every loop counter in a device control block (no host synchronisation).

Semantics the batching fixes (the reference steps ONE env and runs train_step_rnn once per step):
  * one vector step = one env step in every arena, then `updates_per_step` (U) DRQN updates of
    `batch` sequences once the sequence buffer holds > batch * min_episodes_for_training_start
    episodes (:776-777), each on its own sampled batch. U = n keeps the reference's one update per
    env step (the generation controller's setting); U = 1 is the throughput setting;
  * modelB's acting noise is drawn fresh once per vector step and shared by all arenas (the
    reference resets it before each greedy action, :385); the update uses modelB's epsilon buffers
    as that draw left them (train_step_rnn does not reset noise);
  * epsilon decays once per finished episode (:798), applied after the vector step;
  * each episode plays modelA or (p = opponent_pool_ratio) a uniformly drawn pool net (:735-736),
    every opponent in eval mode (:344, :615); both players start each episode from zero (h, c);
  * the sequence buffer keeps the latest `memory_size` episodes of length >= trace_length
    (deque(maxlen), :104, :112-115); their steps live in per-arena rings of `depth` steps. So that
    no sample can reach an overwritten step, a trajectory longer than depth / 2 is not stored and
    an episode leaves once depth / 2 steps have passed since it finished; `ring_depth` sizes depth
    so neither happens at the expected episode lengths, and `check_status` raises / warns if the
    device saw otherwise;
  * max_episode_steps (:751, default 1000): an episode still running after that many steps ends
    (counters, epsilon decay, new opponent, env.reset, zero (h, c)) while its trajectory goes on
    collecting steps until a done, as push_step's current_episode_trajectory does.
Overlap (default): the opponents' act of the next vector step (modelA / pool nets in eval mode) reads
nothing the DRQN update writes, so it runs on a side stream beside the update on part of the chip
and each step's act is modelB's side only (pm_rnn_selfplay_step_overlap); results are bit-identical.
Sharded (world > 1): every rank owns n arenas and its own sequence buffer; the gradient (+ the
contributing-rank count) is summed by one all-reduce per update and every rank applies the
identical clip + Adam step (pongmi.drqn).
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import PM_RNN_NW, PM_TRANS_F, check, ptr, stream_ptr
from .dist import shard_seeds
from .drqn import DRQNLearner
from .env import env_config, env_params
from .rnn import fold, pack_state_dict, unpack_state_dict
from .selfplay import act_chunk


def ring_depth(n, memory_size, mean_len=40, margin=512):
    """Steps per arena ring, a power of two: depth / 2 (the age an episode may reach in the buffer, and
    the longest trajectory stored) covers the span of the newest `memory_size` episodes (~memory_size
    * mean_len / n vector steps) with 50 % headroom, plus `margin` steps for long episodes."""
    need = 2 * (int(1.5 * memory_size * mean_len / max(n, 1)) + margin)
    d = 64
    while d < need:
        d *= 2
    return d


def sharded_rnn_vector_step(L, allreduce, updates):
    """One vector step of a sharded QNetRNN learner as its launch sequence (RNNSelfPlayLearner.step
    for world > 1 with a torch.distributed all-reduce; the Python twin of
    pm_rnn_selfplay_step_sharded, csrc/pm_comm.cpp, whose all-reduce is libpongmi's RCCL call):

      rollout (fold + act + env + sequence store + update 0's batch sample);
      per update u: [sample(u) (u > 0)] + learner.grads() + allreduce(learner.grad) + learner.apply().

    learner.grad is the packed exchange buffer: [0, PM_RNN_NPARAM) this rank's gradient (the
    NoisyLinear sigma slots left zero: sigma gradients are mu gradient x epsilon, formed after the
    sum), [PM_RNN_NPARAM] 1 if the rank contributed (its buffer was ready), [PM_RNN_NPARAM + 1] 1 if a
    hand-off timed out on it (the update is then void on every rank). After the SUM every rank's
    apply divides by the contributing-rank count, forms the sigma gradients, clips on the norm of
    that summed gradient (train_rnn_iterative.py:509, clip_grad_norm_ on the global gradient) and
    takes the identical Adam step (:510-516). `L` needs only these launch methods, so the CPU tests
    drive this same sequence over gloo with oracle-backed shards."""
    L.rollout()
    for u in range(updates):
        if u:
            L.sample(u)
        L.learner.grads()
        allreduce(L.learner.grad)  # one all-reduce per update: 174 984 grads + rank count + void count
        L.learner.apply()


class RNNSelfPlayLearner:
    def __init__(self, env_kw, n_arenas, modelB_state, modelA_state=None, pool_states=(), *, batch=64, trace_length=8,
                 memory_size=200_000, min_episodes_for_training_start=10, depth=None, gamma=0.99, lr=1e-4,
                 epsilon=1.0, min_epsilon=0.05, epsilon_decay=0.999, target_update_interval=2000, pool_ratio=0.4,
                 grad_clip_norm=1.0, episode=0, seed=0, rank=0, world=1, allreduce=None, device=None,
                 updates_per_step=1, max_episode_steps=1000, overlap=True, record_q=False):
        self.lib = _lib.load()
        self.overlap = bool(overlap)
        # The overlapped step acts for the NEXT step's opponents speculatively, reading (h, c) of
        # buffer _cur and writing the other one; _spec: that act is done for the current observations
        # (its input state still intact in buffer 1 - _cur), _stale: the opponents changed since, so it
        # is redone from that state before the next step (bit-identical to the plain step).
        self._cur, self._spec, self._stale = 0, False, False
        self.updates_per_step = int(updates_per_step)
        if self.updates_per_step < 1:
            raise ValueError("updates_per_step must be >= 1")
        self._warned = 0
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise _lib.PongmiError("RNNSelfPlayLearner runs on a ROCm device only")
        self.n, self.T, self.cap = int(n_arenas), int(trace_length), int(memory_size)
        self.world, self.rank = int(world), int(rank)
        if self.world > 1 and allreduce is None:
            raise ValueError("world > 1 needs an allreduce(tensor) callable (torch.distributed.all_reduce)")
        self.allreduce = allreduce
        self.env_cfg = env_config(**env_kw)
        self.depth = int(depth) if depth else ring_depth(self.n, self.cap)
        dev, n = self.device, self.n
        f32 = dict(dtype=torch.float32, device=dev)
        # ---- environment SoA + per-arena bookkeeping
        self.f64 = torch.zeros((7, n), dtype=torch.float64, device=dev)
        self.i32 = torch.zeros((4, n), dtype=torch.int32, device=dev)
        self.opp = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ep_reward = torch.zeros(n, **f32)
        self.ep_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.ep_steps = torch.zeros(n, dtype=torch.int32, device=dev)
        self.reset = torch.ones(n, dtype=torch.uint8, device=dev)
        self.hB, self.cB = (torch.zeros((n, 128), **f32) for _ in range(2))
        self._hAb = [torch.zeros((n, 128), **f32) for _ in range(2)]  # opponents' (h, c): two buffers each
        self._cAb = [torch.zeros((n, 128), **f32) for _ in range(2)]
        self.obsA = torch.zeros((n, 7), **f32)
        self.obsB = torch.zeros((n, 7), **f32)
        self.aA = torch.zeros(n, dtype=torch.int8, device=dev)
        self.aB = torch.zeros(n, dtype=torch.int8, device=dev)
        # ---- sequence buffer
        self.trans = torch.zeros((self.depth, n, PM_TRANS_F), **f32)
        self.seq_eps = torch.zeros((self.cap, 2), dtype=torch.int64, device=dev)
        self.seq_mark = torch.zeros(self.depth, dtype=torch.int64, device=dev)
        self.fin = torch.zeros((((n + 255) // 256) * 256, 2), dtype=torch.int64, device=dev)  # staging
        self.partials = torch.zeros(((n + 255) // 256) * 8, dtype=torch.int64, device=dev)
        self.opp_list = torch.zeros(n, dtype=torch.int32, device=dev)
        self.opp_cnt = torch.zeros(((n + 255) // 256) * (len(pool_states) + 1), dtype=torch.int32, device=dev)
        self.enable = torch.zeros(1, dtype=torch.int32, device=dev)
        # ---- networks
        self.learner = DRQNLearner(modelB_state, batch=batch, T=self.T, gamma=gamma, lr=lr, max_norm=grad_clip_norm,
                                   target_update_interval=target_update_interval, enable=self.enable, device=dev)
        self.batch = self.learner.batch
        self.w_B = torch.zeros(PM_RNN_NW, **f32)
        self.n_pool = len(pool_states)
        self.w_opp = torch.zeros((1 + self.n_pool, PM_RNN_NW), **f32)
        self.set_modelA(modelA_state if modelA_state is not None else modelB_state)
        if self.n_pool:
            pool = torch.stack([pack_state_dict(s, dev) for s in pool_states])
            self.w_opp[1:] = fold(pool, _lib.PM_FOLD_EVAL)  # m_rnn.eval() (:615-617)
        # ---- control block
        c = _lib.RnnCtrl()
        c.epsilon = float(epsilon)
        c.episodes = int(episode)
        self.ctrl = torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8).to(dev)

        sp = _lib.RnnSelfPlay()
        sp.env = env_params(**env_kw)
        sp.st = _lib.EnvState(*[ptr(self.f64[k]) for k in range(7)], *[ptr(self.i32[k]) for k in range(4)])
        for name in ("opp", "ep_reward", "ep_len", "ep_steps", "reset", "w_opp", "w_B", "hA", "cA", "hB", "cB", "obsA",
                     "obsB", "aA", "aB", "trans", "seq_eps", "seq_mark", "fin", "partials", "opp_list", "opp_cnt",
                     "enable", "ctrl"):
            setattr(sp, name, ptr(getattr(self, name)))
        sp.paramsB = ptr(self.learner.params)
        # record_q: the act also writes the Q values each player chose from ([n, 3] each, qA / qB), for
        # parity checks of the acting decision beside the actions of the same launch
        self.qA = torch.zeros((n, 3), **f32) if record_q else None
        self.qB = torch.zeros((n, 3), **f32) if record_q else None
        sp.qA, sp.qB = (ptr(self.qA), ptr(self.qB)) if record_q else (None, None)
        sp.n, sp.n_pool, sp.depth, sp.T = n, self.n_pool, self.depth, self.T
        sp.max_steps = int(max_episode_steps or 0)
        p_pool = pool_ratio if self.n_pool else 0.0
        sp.chunk_A = act_chunk(1.0 - p_pool, cap=2048)
        sp.chunk_P = act_chunk(p_pool / self.n_pool, cap=2048) if self.n_pool else 256
        sp.seq_cap = self.cap
        sp.min_episodes = int(self.batch * min_episodes_for_training_start)
        sp.min_epsilon, sp.epsilon_decay, sp.pool_ratio = float(min_epsilon), float(epsilon_decay), float(pool_ratio)
        self.seed = int(seed)
        sp.seed_env, sp.seed_net = shard_seeds(self.seed, self.rank)
        self.sp = sp
        self.side = torch.cuda.Stream(device=dev)  # the overlapped step's opponent act (beside the update)
        check(self.lib.pm_rnn_selfplay_init(ctypes.byref(sp), stream_ptr()), "pm_rnn_selfplay_init")

    # ------------------------------------------------------------------ stepping
    @property
    def hA(self):
        """The opponents' hidden state after the latest act for them, [n, 128]."""
        return self._hAb[self._cur]

    @property
    def cA(self):
        return self._cAb[self._cur]

    def _opp_buffers(self, src, dst):
        """The opponents' act reads (h, c) from buffer src (None: dst, in place) and writes buffer dst."""
        sp = self.sp
        sp.hA, sp.cA = ptr(self._hAb[dst]), ptr(self._cAb[dst])
        sp.hA_in = None if src is None else ptr(self._hAb[src])
        sp.cA_in = None if src is None else ptr(self._cAb[src])

    def _prepare_overlap(self):
        """Before an overlapped step: the opponents' actions for the current observations (the last
        step's speculative act, redone from its saved input state if the opponents changed since, or a
        first act in place), then point the act at the other buffer."""
        if not self._spec or self._stale:
            self._opp_buffers(1 - self._cur if self._spec else None, self._cur)
            check(self.lib.pm_rnn_selfplay_act_part(ctypes.byref(self.sp), _lib.PM_ACT_A, stream_ptr()),
                  "pm_rnn_selfplay_act_part")
        self._opp_buffers(self._cur, 1 - self._cur)

    def _commit_overlap(self):
        self._cur = 1 - self._cur
        self._opp_buffers(None, self._cur)
        self._spec, self._stale = True, False

    def act(self):
        """modelB fold with fresh noise + both players' act (in place)."""
        self._spec = False
        check(self.lib.pm_rnn_selfplay_act(ctypes.byref(self.sp), stream_ptr()), "pm_rnn_selfplay_act")

    def act_part(self, part):
        """PM_ACT_B: modelB's fold (fresh noise) + act; PM_ACT_A: the opponents' act; PM_ACT_ALL: both
        (in place)."""
        if part != _lib.PM_ACT_B:
            self._spec = False
        check(self.lib.pm_rnn_selfplay_act_part(ctypes.byref(self.sp), int(part), stream_ptr()),
              "pm_rnn_selfplay_act_part")

    def finish_overlap(self):
        """The overlapped step after act_part(PM_ACT_B): env + sample, the next step's opponent act on
        the side stream beside the updates, join."""
        self._prepare_overlap()
        check(self.lib.pm_rnn_selfplay_finish_overlap(ctypes.byref(self.sp), ctypes.byref(self.learner.desc),
                                                      self.updates_per_step, self.side.cuda_stream, stream_ptr()),
              "pm_rnn_selfplay_finish_overlap")
        self._commit_overlap()

    def env_step(self):
        """env tick + sequence store + counters + batch sample / enable flag."""
        self._spec = False
        check(self.lib.pm_rnn_selfplay_env(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), stream_ptr()),
              "pm_rnn_selfplay_env")

    def rollout(self):
        """fold + act + env + sequence store + batch sample (no update). After an overlapped step the
        opponents already acted for the current observations (speculatively, into buffer _cur): acting
        for them again would advance their LSTM state twice on one observation, so the rollout then
        acts for modelB only (the speculative act redone first if the opponents changed since)."""
        if self._spec:
            if self._stale:
                self._opp_buffers(1 - self._cur, self._cur)
                check(self.lib.pm_rnn_selfplay_act_part(ctypes.byref(self.sp), _lib.PM_ACT_A, stream_ptr()),
                      "pm_rnn_selfplay_act_part")
                self._opp_buffers(None, self._cur)
                self._stale = False
            self.act_part(_lib.PM_ACT_B)
            self.env_step()
            return
        self._spec = False
        check(self.lib.pm_rnn_selfplay_rollout(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), stream_ptr()),
              "pm_rnn_selfplay_rollout")

    def sample(self, u):
        """Batch of update u >= 1 of the current vector step (update 0's is drawn by env_step)."""
        check(self.lib.pm_rnn_selfplay_sample(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), int(u),
                                              stream_ptr()), "pm_rnn_selfplay_sample")

    def step(self):
        """One vector step (n env-steps on this rank) and its `updates_per_step` DRQN updates when
        enabled."""
        U = self.updates_per_step
        comm = getattr(self.allreduce, "pm_comm", None)
        if comm is not None and self.overlap:  # sharded + overlapped: one call, all-reduce in stream
            self._prepare_overlap()
            check(self.lib.pm_rnn_selfplay_step_sharded_overlap(ctypes.byref(self.sp), ctypes.byref(self.learner.desc),
                                                                comm, U, self.side.cuda_stream, stream_ptr()),
                  "pm_rnn_selfplay_step_sharded_overlap")
            self._commit_overlap()
            return
        if comm is not None:  # pongmi.dist.NativeComm: the sharded step as one call, all-reduce in stream
            self._spec = False
            check(self.lib.pm_rnn_selfplay_step_sharded(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), comm,
                                                        U, stream_ptr()), "pm_rnn_selfplay_step_sharded")
            return
        if self.world == 1 and self.overlap:  # the next step's opponent act beside this step's update
            self._prepare_overlap()
            check(self.lib.pm_rnn_selfplay_step_overlap(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), U,
                                                        self.side.cuda_stream, stream_ptr()),
                  "pm_rnn_selfplay_step_overlap")
            self._commit_overlap()
            return
        self._spec = False
        if self.world == 1:
            check(self.lib.pm_rnn_selfplay_step_multi(ctypes.byref(self.sp), ctypes.byref(self.learner.desc), U,
                                                      stream_ptr()), "pm_rnn_selfplay_step_multi")
            return
        sharded_rnn_vector_step(self, self.allreduce, U)

    def check_status(self, c=None, log=print):
        """Device error bits (pm_rnn_ctrl.status): bit 0 (a sample read an overwritten ring step) means
        corrupted training data and raises; bits 1 / 2 (episodes evicted by age / a trajectory longer
        than depth / 2 dropped: `depth` is too small for the episode lengths seen) warn once each. The
        DRQN learner's pm_drqn_stats.status is checked too: a timed-out hand-off (a voided update)
        raises."""
        st = int((c or self.counters())["status"])
        if st & 1:
            raise _lib.PongmiError(f"RNN sequence buffer: a sampled step had been overwritten (status {st}); "
                                   f"depth {self.depth} is too small")
        self.learner.check_status()  # the DRQN update's own word (pm_drqn_stats.status): a void update raises
        new = st & 6 & ~self._warned
        if new & 2:
            log(f"[WARNING] sequence buffer: episodes older than depth/2 = {self.depth // 2} steps were evicted "
                f"before {self.cap} newer ones; raise depth (ring_depth) for longer episodes")
        if new & 4:
            log(f"[WARNING] sequence buffer: a trajectory longer than depth/2 = {self.depth // 2} steps was not "
                f"stored; raise depth for longer rallies")
        self._warned |= new
        return st

    # ------------------------------------------------------------------ state readout (syncs)
    def counters(self):
        c = _lib.RnnCtrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        out = {k: getattr(c, k) for k, _ in _lib.RnnCtrl._fields_}
        out["train_steps"] = self.learner.stats()["steps"]
        return out

    def set_epsilon(self, eps):
        c = _lib.RnnCtrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        c.epsilon = float(eps)
        self.ctrl.copy_(torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8))

    def set_modelA(self, state):
        """Opponent slot 0: modelA, frozen and in eval mode (train_rnn_iterative.py:343-344)."""
        self._stale = self._spec
        self.paramsA = pack_state_dict(state, self.device)
        self.w_opp[0] = fold(self.paramsA, _lib.PM_FOLD_EVAL)[0]

    def modelB_state_dict(self):
        return unpack_state_dict(self.learner.params)

    def targetB_state_dict(self):
        return unpack_state_dict(self.learner.target)

    def modelA_state_dict(self):
        return unpack_state_dict(self.paramsA)

    # ------------------------------------------------------------------ generation controller hooks
    def reset_B(self, state, epsilon=1.0, reset_train_steps=True):
        """modelB <- state with a new Adam, targetB <- modelB, epsilon reset (reset_model_b_for_new_attempt,
        train_rnn_iterative.py:669-702; also the new-generation start, :711-722, which keeps
        train_steps_count: reset_train_steps=False). The sequence buffer is kept, as there."""
        self.learner.load_params(state)
        self.learner.new_optimizer()
        if reset_train_steps:
            self.learner.set_train_steps(0)
        self.set_epsilon(epsilon)

    def add_pool_model(self, state):
        """pool_models.append(net in eval mode) (:855-859): opponent slot n_pool + 1 for later draws."""
        self._stale = self._spec
        w = fold(pack_state_dict(state, self.device), _lib.PM_FOLD_EVAL)
        self.w_opp = torch.cat([self.w_opp, w], 0).contiguous()
        self.n_pool += 1
        n = self.n
        self.opp_cnt = torch.zeros(((n + 255) // 256) * (self.n_pool + 1), dtype=torch.int32, device=self.device)
        sp = self.sp
        sp.w_opp, sp.opp_cnt, sp.n_pool = ptr(self.w_opp), ptr(self.opp_cnt), self.n_pool
        p_pool = sp.pool_ratio
        sp.chunk_A = act_chunk(1.0 - p_pool, cap=2048)
        sp.chunk_P = act_chunk(p_pool / self.n_pool, cap=2048)
        self._rebuild_lists()

    def _rebuild_lists(self):
        """Per-block opponent lists for the current opponent ids (the env kernel keeps them after this)."""
        opp = self.opp.cpu().numpy()
        nn = self.n_pool + 1
        neb = (self.n + 255) // 256
        lst = np.zeros(self.n, np.int32)
        cnt = np.zeros(neb * nn, np.int32)
        for e in range(neb):
            ids = opp[e * 256:(e + 1) * 256]
            off = 0
            for k in range(nn):
                sel = np.nonzero(ids == k)[0] + e * 256
                lst[e * 256 + off:e * 256 + off + len(sel)] = sel
                cnt[e * nn + k] = (off << 16) | len(sel)
                off += len(sel)
        self.opp_list.copy_(torch.from_numpy(lst))
        self.opp_cnt.copy_(torch.from_numpy(cnt))

    def set_counters(self, **kw):
        c = _lib.RnnCtrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        for k, v in kw.items():
            setattr(c, k, v)
        self.ctrl.copy_(torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8))

    def episodes(self):
        """The stored episodes, oldest first: (arena, first step, length) int64 [seq_size, 3] (host)."""
        c = self.counters()
        size, count = c["seq_size"], c["seq_count"]
        raw = self.seq_eps.cpu()
        idx = (torch.arange(count - size, count) % self.cap)
        e = raw[idx]
        return torch.stack([e[:, 0] & 0xFFFFFFFF, e[:, 1], e[:, 0] >> 32], 1)
