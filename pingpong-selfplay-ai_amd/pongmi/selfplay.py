"""The batched self-play DQN learner: scripts/train_iterative.py's hot loop (:239-245) for n arenas
per device, as four libpongmi launches sequences per vector step (rollout / learn / [all-reduce] /
apply) on one stream, with every loop counter in a device control block.

Semantics the batching fixes (the reference steps ONE env and updates once per env step):
  * one vector step = one env step in every arena, then `updates_per_step` (U) PER updates of
    `batch`. The reference's replay ratio is one update per pushed transition (:243-244): U = n
    keeps it (the generation controllers do, with a few hundred arenas); U = 1, the throughput
    setting the bench measures, trains once per n transitions. With U > 1, update 0 samples with
    the step's push pending (as U = 1) and updates 1..U-1 resample the replay after it; every
    update advances frame_idx (beta), the noise counter, train_steps and the target sync;
  * NoisyNet acting noise is fresh per vector step and shared by all arenas (reset_noise per
    select_action_B, :125), the update draws its own fresh noise (:142);
  * epsilon decays once per finished episode: eps <- max(min_eps, eps * decay^D) for the D
    episodes finished in a vector step (:261);
  * each episode independently plays modelA or (p = opponent_pool_ratio) a uniformly drawn pool
    net (:235-236);
  * pushes of a vector step all receive the max priority held before the step (:57): the running
    maximum when U = 1 (exact, since n > batch pushes survive the scatter), the array maximum
    recomputed by pm_selfplay_commit when U > 1.
Sharded (world > 1): every rank owns n arenas and its own replay; `sp.grad` (520 head grads +
counters) is summed by one all-reduce per update and every rank applies the identical Adam step.
`allreduce` is a callable on that buffer (torch.distributed.all_reduce), or a pongmi.dist.NativeComm:
then a vector step is one library call with the RCCL all-reduce on the learner's stream.
"""
import ctypes

import numpy as np
import torch

from . import _lib, checkpoint
from ._lib import (PM_GRAD_EPISODES, PM_GRAD_LEN, PM_GRAD_UPDATED, PM_QNET_NHEAD, PM_QNET_NP, PM_QNET_NW,  # noqa: F401
                   PM_TRANS_F, check, ptr, stream_ptr)
from .dist import shard_seeds, splitmix64  # noqa: F401
from .env import env_config, env_params
from .qnet import HEAD_KEYS, fold, pack_state_dict, unpack_state_dict


def act_chunk(p, rows=96, cap=4096, lo=256):
    """Arenas per act chunk of an opponent played with probability p: the smallest power of two
    >= `lo` expected to hold >= `rows` of its arenas (so its 32-row MFMA tiles are mostly full).
    Multiples of 256 let the act kernel read the env kernel's per-block opponent lists."""
    if p <= 0:
        return cap
    c = lo
    while c < cap and c * p < rows:
        c *= 2
    return c


def sharded_vector_step(L, allreduce, updates):
    """One vector step of a (sharded) learner as its launch sequence: the Python twin of
    pm_selfplay_step_sharded (csrc/pm_comm.cpp), for an `allreduce` callable on the packed buffer
    (torch.distributed, gloo in the CPU tests) instead of the library's RCCL communicator.

      overlap: [act(A) if the opponents' actions are stale] + actenv, else rollout;
      per update u: [resample (u > 0)] + learn_ex(u = 0: FIRST (| LAST when U = 1), with the next
        step's side-A act when overlapped) + allreduce(L.grad) + apply_ex(same mode);
      U > 1: commit.

    L.grad is the packed exchange buffer (include/pongmi.h PM_GRAD_*): [0, 520) the shard's head
    gradients, [PM_GRAD_EPISODES] its finished episodes (update 0), [PM_GRAD_UPDATED] 1 if it trained;
    after the SUM every rank's apply uses grads / world and decays epsilon by the summed episodes.
    `allreduce` None: a single learner (world 1, unfused apply). `L` needs only the learner's launch
    methods, so the CPU tests drive this same sequence with oracle-backed shards."""
    if L.overlap:
        if not L._aA_ready:
            L.act(_lib.PM_ACT_A)
        L.actenv()
    else:
        L.rollout()
    for u in range(updates):
        mode = (_lib.PM_UPD_FIRST | (_lib.PM_UPD_LAST if updates == 1 else 0)) if u == 0 else 0
        if u:
            L.resample()
        L.learn_ex(mode, act_next=L.overlap and u == 0)
        if allreduce is not None:
            allreduce(L.grad)
        L.apply_ex(mode)
    if updates > 1:
        L.commit()


class SelfPlayLearner:
    def __init__(self, env_kw, n_arenas, modelB_state, modelA_state=None, pool_states=(), *, batch=256,
                 memory_size=1_000_000, gamma=0.99, lr=2.5e-4, epsilon=0.02, min_epsilon=0.02, epsilon_decay=0.995,
                 target_update_interval=1000, pool_ratio=0.33, alpha=0.6, beta_start=0.4, beta_frames=100000,
                 episode=0, seed=0, rank=0, world=1, allreduce=None, device=None, modelA_noisy=True,
                 fuse_apply=True, overlap=True, updates_per_step=1, features_ahead=True, learn_multi=True):
        self.lib = _lib.load()
        self.updates_per_step = int(updates_per_step)
        if self.updates_per_step < 1:
            raise ValueError("updates_per_step must be >= 1")
        self.overlap = bool(overlap)
        self._aA_ready = False
        self.device = torch.device(device if device is not None else "cuda")
        if self.device.type != "cuda":
            raise _lib.PongmiError("SelfPlayLearner runs on a ROCm device only")
        self.n, self.batch, self.cap = int(n_arenas), int(batch), int(memory_size)
        self.world, self.rank = int(world), int(rank)
        if self.world > 1 and allreduce is None:
            raise ValueError("world > 1 needs an allreduce(tensor) callable (torch.distributed.all_reduce)")
        self.allreduce = allreduce
        self.env_cfg = env_config(**env_kw)
        dev, n = self.device, self.n
        f32 = dict(dtype=torch.float32, device=dev)

        # ---- environment SoA + per-arena bookkeeping
        self.f64 = torch.zeros((7, n), dtype=torch.float64, device=dev)
        self.i32 = torch.zeros((4, n), dtype=torch.int32, device=dev)
        self.opp = torch.zeros(n, dtype=torch.int32, device=dev)
        self.opp_list = torch.zeros(n, dtype=torch.int32, device=dev)
        self.opp_cnt = torch.zeros(((n + 255) // 256) * (len(pool_states) + 1), dtype=torch.int32, device=dev)
        self.ep_reward = torch.zeros(n, **f32)
        # ---- networks
        self.paramsB = pack_state_dict(modelB_state, dev)
        self.paramsT = self.paramsB.clone()
        self.adam_m = torch.zeros(PM_QNET_NHEAD, **f32)
        self.adam_v = torch.zeros(PM_QNET_NHEAD, **f32)
        self.w_B = torch.zeros(PM_QNET_NW, **f32)
        self.n_pool = len(pool_states)
        self.w_opp = torch.zeros((1 + self.n_pool, PM_QNET_NW), **f32)
        self.modelA_noisy = modelA_noisy
        self.set_modelA(modelA_state if modelA_state is not None else modelB_state)
        if self.n_pool:
            pool = torch.stack([pack_state_dict(s, dev) for s in pool_states])
            self.w_opp[1:] = fold(pool, _lib.PM_FOLD_EVAL)  # pool nets are .eval() (:205)
        # ---- replay + learner scratch
        self.trans = torch.zeros((self.cap, PM_TRANS_F), **f32)
        self.prios = torch.zeros(self.cap, **f32)
        self.per_work = torch.zeros(max(self.lib.pm_per_work_bytes(self.cap), 256), dtype=torch.uint8, device=dev)
        self.idx = torch.zeros(self.batch, dtype=torch.int64, device=dev)
        self.isw = torch.zeros(self.batch, **f32)
        self.grad = torch.zeros(PM_GRAD_LEN, **f32)  # the packed exchange buffer (include/pongmi.h PM_GRAD_*)
        self.partials = torch.zeros(((n + 255) // 256) * 8, dtype=torch.int64, device=dev)
        # + the push-row hand-off rows and flag, the tree-refresh epoch and granules (pongmi.h, ABI 21)
        self.hfeat = torch.zeros((4 * self.batch + 8, 80), **f32)
        self.learn_heads = torch.zeros(3 * 264, **f32)
        self.obsA = torch.zeros((n, 7), **f32)
        self.obsB = torch.zeros((n, 7), **f32)
        self.aA = torch.zeros(n, dtype=torch.int8, device=dev)
        self.aB = torch.zeros(n, dtype=torch.int8, device=dev)
        # modelB's hidden features of the next step's observations, computed with the opponents' act
        # (features are frozen: only the heads train), so the fused act + env kernel evaluates heads only
        self.featB = torch.zeros(((n + 31) // 32) * 2048, **f32) if features_ahead else None
        # U > 1: ReLU(modelB's features) of every replay row's s, stored at push time, so updates 1..U-1
        # of a vector step run as one single-workgroup launch (k_learn_multi; 256 B per replay row)
        use_frow = learn_multi and self.updates_per_step > 1 and features_ahead and self.overlap and world == 1
        self.frow = torch.zeros((self.cap, 64), **f32) if use_frow else None
        self._frow_wait = 0  # vector steps pushed through actenv still needed before frow is current
        # ---- control block
        c = _lib.Ctrl()
        c.epsilon = float(epsilon)
        c.max_prio = 1.0
        c.episodes = int(episode)
        self.ctrl = torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8).to(dev)

        self.seed = int(seed)
        sp = _lib.SelfPlay()
        sp.env = env_params(**env_kw)
        sp.st = _lib.EnvState(*[ptr(self.f64[k]) for k in range(7)], *[ptr(self.i32[k]) for k in range(4)])
        for name in ("opp", "ep_reward", "w_opp", "paramsB", "paramsT", "w_B", "adam_m", "adam_v", "trans", "prios",
                     "per_work", "idx", "isw", "grad", "partials", "obsA", "obsB", "aA", "aB", "hfeat", "learn_heads",
                     "ctrl", "opp_list", "opp_cnt"):
            setattr(sp, name, ptr(getattr(self, name)))
        sp.featB = ptr(self.featB)
        sp.frow = ptr(self.frow)
        sp.frow_ready = int(self.frow is not None)
        sp.n, sp.n_pool, sp.batch, sp.world, sp.cap = n, self.n_pool, self.batch, self.world, self.cap
        sp.fuse_apply = int(bool(fuse_apply) and self.world == 1)
        p_pool = pool_ratio if self.n_pool else 0.0
        sp.chunk_A = act_chunk(1.0 - p_pool)
        sp.chunk_P = act_chunk(p_pool / self.n_pool) if self.n_pool else 256
        sp.gamma, sp.alpha, sp.lr = gamma, alpha, lr
        sp.beta1, sp.beta2, sp.adam_eps = 0.9, 0.999, 1e-8
        sp.min_epsilon, sp.epsilon_decay, sp.pool_ratio, sp.beta_start = min_epsilon, epsilon_decay, pool_ratio, beta_start
        sp.beta_frames, sp.target_update_interval = int(beta_frames), int(target_update_interval)
        sp.seed_env, sp.seed_net = shard_seeds(self.seed, self.rank)
        self.sp = sp
        self.hparams = dict(gamma=gamma, lr=lr, min_epsilon=min_epsilon, epsilon_decay=epsilon_decay,
                            target_update_interval=target_update_interval, pool_ratio=pool_ratio, alpha=alpha,
                            beta_start=beta_start, beta_frames=beta_frames)
        check(self.lib.pm_selfplay_init(ctypes.byref(sp), stream_ptr()), "pm_selfplay_init")

    # ------------------------------------------------------------------ stepping
    # `_aA_ready`: sp.aA holds the opponents' actions for the current observations (computed by a
    # side-A act, or by the extra blocks of the previous step's learner launch), and sp.featB modelB's
    # features of them (computed by the same launches). Anything that changes the observations,
    # opponent ids, opponent weights or modelB's feature layers clears it.
    def _frow_pushed(self, through_actenv):
        """Bookkeeping of sp.frow_ready: a push through k_env (rollout / env_step) stores no features, so
        k_learn_multi waits until those rows have left the ring (cap / n pushes through actenv)."""
        if self.frow is None:
            return
        if through_actenv:
            self._frow_wait = max(0, self._frow_wait - 1)
        else:
            self._frow_wait = -(-self.cap // self.n) + 1
        self.sp.frow_ready = int(self._frow_wait == 0)

    def rollout(self):
        self._aA_ready = False
        self._frow_pushed(False)
        check(self.lib.pm_selfplay_rollout(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_rollout")

    def act(self, part=_lib.PM_ACT_ALL):
        check(self.lib.pm_selfplay_act_part(ctypes.byref(self.sp), int(part), stream_ptr()), "pm_selfplay_act_part")
        if part != _lib.PM_ACT_B:
            self._aA_ready = True

    def actenv(self):
        """act(PM_ACT_B) + env_step fused into one launch (bit-identical)."""
        self._aA_ready = False
        self._frow_pushed(True)
        check(self.lib.pm_selfplay_actenv(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_actenv")

    def env_step(self):
        self._aA_ready = False
        self._frow_pushed(False)
        check(self.lib.pm_selfplay_env(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_env")

    def learn(self, act_next=False):
        """train_step; with act_next the same launch also computes the next vector step's opponent
        actions (after env_step: for the observations it wrote)."""
        if act_next:
            check(self.lib.pm_selfplay_learn_act(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_learn_act")
            self._aA_ready = True
        else:
            check(self.lib.pm_selfplay_learn(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_learn")

    def apply(self):
        check(self.lib.pm_selfplay_apply(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_apply")

    def learn_ex(self, mode, act_next=False):
        check(self.lib.pm_selfplay_learn_ex(ctypes.byref(self.sp), int(mode), int(bool(act_next)), stream_ptr()),
              "pm_selfplay_learn_ex")
        if act_next:
            self._aA_ready = True

    def apply_ex(self, mode):
        check(self.lib.pm_selfplay_apply_ex(ctypes.byref(self.sp), int(mode), stream_ptr()), "pm_selfplay_apply_ex")

    def resample(self):
        """The PER sample + batch forward of updates 1..U-1 of a vector step."""
        check(self.lib.pm_selfplay_resample(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_resample")

    def commit(self):
        """Close a vector step of U > 1 updates: max_prio = max(prios), next-push tree nodes, counters."""
        check(self.lib.pm_selfplay_commit(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_commit")

    def _step_sharded(self, comm):
        """The sharded step as one library call (pongmi.dist.NativeComm): the all-reduce rides the
        learner's stream between k_learn and k_adam (same results as the Python sequence)."""
        self._frow_pushed(True)
        if not self._aA_ready:
            self.act(_lib.PM_ACT_A)
        check(self.lib.pm_selfplay_step_sharded(ctypes.byref(self.sp), comm, self.updates_per_step, stream_ptr()),
              "pm_selfplay_step_sharded")
        self._aA_ready = True

    def _step_multi(self):
        U = self.updates_per_step
        if self.world == 1 and self.overlap:
            if not self._aA_ready:
                self.act(_lib.PM_ACT_A)
            self._frow_pushed(True)
            check(self.lib.pm_selfplay_step_multi(ctypes.byref(self.sp), U, stream_ptr()), "pm_selfplay_step_multi")
            self._aA_ready = True
            return
        sharded_vector_step(self, self.allreduce if self.world > 1 else None, U)

    def step(self):
        """One vector step (n env-steps on this rank) and its `updates_per_step` updates. With
        `overlap` the opponents' act for the next step runs inside the learner's launch
        (bit-identical results)."""
        comm = getattr(self.allreduce, "pm_comm", None)
        if comm is not None and self.overlap and not self.sp.fuse_apply:
            self._step_sharded(comm)
            return
        if self.updates_per_step > 1:
            self._step_multi()
            return
        if self.world > 1:
            sharded_vector_step(self, self.allreduce, 1)
            return
        if not self.overlap:
            self._frow_pushed(False)
            check(self.lib.pm_selfplay_step(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_step")
            return
        if not self._aA_ready:
            self.act(_lib.PM_ACT_A)
        self._frow_pushed(True)
        check(self.lib.pm_selfplay_step_overlap(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_step_overlap")
        self._aA_ready = True

    # ------------------------------------------------------------------ state readout (syncs)
    def counters(self):
        c = _lib.Ctrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        return {k: getattr(c, k) for k, _ in _lib.Ctrl._fields_ if not k.startswith("_")}

    def check_status(self, c=None):
        """Device error bits (pm_ctrl.status): bit 0 = an update's push-row hand-off inside k_learn
        timed out (its push rows were not computed: that update is void); bit 1 = an update scattered
        a NaN priority (the loss diverged; the reference's sampler would raise on the NaN
        probabilities); bit 2 = k_learn's tree-refresh block timed out waiting for the learner (the
        sum tree is stale until repair_tree). Raises on any of them; bit 3 (a stale tree was
        repaired) is informational."""
        st = int((c or self.counters())["status"]) & 7
        if st:
            raise _lib.PongmiError(f"self-play learner: device status {st} (bit 0: push-row hand-off timed out; "
                                   f"bit 1: NaN priority scattered; bit 2: tree refresh timed out)")

    def repair_tree(self, c=None):
        """If a tree-refresh timeout left the PER sum tree stale (status bit 2), rebuild it from the
        priorities (pm_selfplay_repair_tree: bit 2 -> bit 3). Returns whether it did. The generation
        controllers call it at every episode check (pongmi.generations._play_episodes)."""
        if not int((c or self.counters())["status"]) & 4:
            return False
        check(self.lib.pm_selfplay_repair_tree(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_repair_tree")
        return True

    def set_epsilon(self, eps):
        c = _lib.Ctrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        c.epsilon = float(eps)
        self.ctrl.copy_(torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8))

    def modelB_state_dict(self):
        return unpack_state_dict(self.paramsB)

    def targetB_state_dict(self):
        return unpack_state_dict(self.paramsT)

    def set_modelA(self, state):
        """Opponent slot 0. modelA is never put in eval() by the reference (train_iterative.py:90-92),
        so it acts with its frozen epsilon buffers: W = mu + sigma*eps."""
        self._aA_ready = False
        self.paramsA = pack_state_dict(state, self.device)
        self.w_opp[0] = fold(self.paramsA, _lib.PM_FOLD_TRAIN if self.modelA_noisy else _lib.PM_FOLD_EVAL)[0]

    def modelA_state_dict(self):
        return unpack_state_dict(self.paramsA)

    def optimizer_state_dict(self):
        """torch.optim.Adam state_dict for the 8 head tensors (train_iterative.py:101-104)."""
        shapes = [(1, 64), (1,), (1, 64), (1,), (3, 64), (3,), (3, 64), (3,)]
        return checkpoint.adam_state_dict(shapes, self.adam_m, self.adam_v, self.counters()["train_steps"],
                                          self.hparams["lr"])

    def reset_B(self, state, epsilon=1.0):
        """reset_B (train_iterative.py:213-224): fresh modelB from `state`, new Adam, empty replay,
        epsilon 1.0, target = modelB, train_steps = frame_idx = 0."""
        self.paramsB.copy_(pack_state_dict(state, self.device))
        self.paramsT.copy_(self.paramsB)
        self.adam_m.zero_()
        self.adam_v.zero_()
        self.prios.zero_()
        self.per_work.zero_()  # priority block sums are maintained incrementally
        c = _lib.Ctrl.from_buffer_copy(bytes(self.ctrl.cpu().numpy().tobytes()))
        c.pos = c.size = c.train_steps = c.frame_idx = 0
        c.max_prio = 1.0
        c.epsilon = float(epsilon)
        self.ctrl.copy_(torch.frombuffer(bytearray(bytes(c)), dtype=torch.uint8))
        self.prepare()
        if self.frow is not None:  # the replay is empty: every row k_learn_multi can reach is pushed from now
            self._frow_wait = 0
            self.sp.frow_ready = 1

    def prepare(self):
        """Re-derive acting weights / next-update heads after the host replaced parameters. modelB's
        feature layers may have changed, so the stored row features (frow) wait for a turn of the ring."""
        self._aA_ready = False
        self._frow_pushed(False)
        check(self.lib.pm_selfplay_prepare(ctypes.byref(self.sp), stream_ptr()), "pm_selfplay_prepare")


HEAD_NAMES = HEAD_KEYS
__all__ = ["SelfPlayLearner", "sharded_vector_step", "splitmix64", "HEAD_NAMES", "PM_QNET_NP", "PM_GRAD_EPISODES",
           "PM_GRAD_UPDATED", "PM_GRAD_LEN"]
