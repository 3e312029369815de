"""Host side of K9 (pm_rollout, csrc/pm_rollout.hip): inference-only self-play, K vector steps per launch.

BASELINE configs[1]: the rollout of scripts/train_iterative.py:239-242 with the learner switched off
— modelA greedy on its folded weights, modelB epsilon-greedy with fresh NoisyNet noise every vector
step (select_action_B's reset_noise, :125), PongEnv2P autoreset — for n arenas in lockstep. One
launch runs `steps` vector steps with every arena held in registers; the result is bit-identical to
`steps` repetitions of

    w_B = qnet.fold(paramsB, PM_FOLD_TRAIN_FRESH, seed=seed_net, counter=c)
    aA, aB = qnet.act(wA, None, w_B, env.obsA, env.obsB, epsilon, seed=env.seed, counter=c)
    env.step(aA, aB)                       # autoreset, step-keyed serves: env.counter == c

with c = env.counter (tests/test_gpu_rollout.py). The rollout advances env.counter by `steps`, and
leaves env.obsA / env.obsB holding the observations after the last step; rewards / done / term_obs
of the last step are not produced (no learner consumes them).

With `replay=` (a pongmi.replay.DeviceReplay) the same launch is §8f3's collecting rollout
(pm_rollout_push): every vector step also pushes its n transitions into the ring as the training
loop's memory.push((oB, aB, rB, nB, done)) (:242-243) — the rows go from registers to the ring, and
the launch leaves the PER sum tree current — with ep_reward carried per arena (:245) and the stats
gaining the loop's episode wins (ep_reward > 0, :247) and reward sum.
"""
import torch

from . import _lib
from ._lib import PM_QNET_NP, PM_QNET_NW, PM_ROLL_HEADS, check, ptr, require_device, stream_ptr
from .env import ctypes_ref

STATS = ("episodes", "wins_B", "points_A", "points_B")
STATS_PUSH = STATS + ("wins_B_episode", "reward_B")


class SelfPlayRollout:
    """configs[1]'s workload on a PongEnv2PBatch: modelA (effective weights wA, PM_QNET_NW) against
    modelB (packed parameters paramsB, PM_QNET_NP; NoisyNet heads refolded per vector step).

    run(steps) -> dict of STATS accumulated over the call (host ints; reading them synchronises),
    or the device tensor with sync=False."""

    def __init__(self, env, wA, paramsB, epsilon=0.02, seed_net=0):
        self.lib = _lib.load()
        if env.inject is not None:
            raise _lib.PongmiError("SelfPlayRollout uses production (Philox) serves: the env has a serve table")
        if not env.autoreset:
            raise _lib.PongmiError("SelfPlayRollout needs an autoreset env (the rollout never stops an arena)")
        self.env = env
        self.wA = _weights(wA, PM_QNET_NW, "wA", env.device)
        self.paramsB = _weights(paramsB, PM_QNET_NP, "paramsB", env.device)
        self.epsilon = float(epsilon)
        self.seed_net = int(seed_net) & 0xFFFFFFFFFFFFFFFF
        from .qnet import fold
        # modelB's feature layers (its heads are refolded inside the launch every vector step)
        self.wB = fold(self.paramsB, _lib.PM_FOLD_EVAL).reshape(-1)
        self.heads = torch.empty(0, dtype=torch.float32, device=env.device)
        self.stats = torch.zeros(len(STATS_PUSH), dtype=torch.int64, device=env.device)
        # collecting: ep_reward of each arena's running episode (zero it if the env is reset elsewhere)
        self.ep_reward = torch.zeros(env.n, dtype=torch.float32, device=env.device)

    def set_paramsB(self, paramsB):
        """New modelB parameters (e.g. after a generation's training)."""
        from .qnet import fold
        self.paramsB = _weights(paramsB, PM_QNET_NP, "paramsB", self.env.device)
        self.wB = fold(self.paramsB, _lib.PM_FOLD_EVAL).reshape(-1)

    def reserve(self, steps):
        """Allocate the heads workspace for launches of up to `steps` vector steps ahead of time."""
        if self.heads.numel() < int(steps) * PM_ROLL_HEADS:
            self.heads = torch.empty(int(steps) * PM_ROLL_HEADS, dtype=torch.float32, device=self.env.device)

    def run(self, steps, sync=True, replay=None):
        """replay: None (inference only, pm_rollout) or a DeviceReplay the launch pushes every step's
        transitions into (pm_rollout_push; steps * n <= replay.cap)."""
        steps = int(steps)
        if steps < 0:
            raise ValueError("steps must be >= 0")
        self.reserve(steps)
        self.stats.zero_()
        env = self.env
        names = STATS
        if replay is None:
            check(self.lib.pm_rollout(ctypes_ref(env.params), ctypes_ref(env.state), ptr(self.wA), ptr(self.wB),
                                      ptr(self.paramsB), self.epsilon, env.seed, self.seed_net, env.counter, steps,
                                      ptr(self.heads), ptr(env.obsA), ptr(env.obsB), ptr(self.stats), env.n,
                                      stream_ptr()), "pm_rollout")
        else:
            names = STATS_PUSH
            rp = _lib.RollReplay(trans=ptr(replay.trans), prios=ptr(replay.prios), per_work=ptr(replay.work),
                                 ep_reward=ptr(self.ep_reward), pos=replay.pos, cap=replay.cap,
                                 prio=replay.push_prio(), alpha=replay.alpha)
            check(self.lib.pm_rollout_push(ctypes_ref(env.params), ctypes_ref(env.state), ptr(self.wA), ptr(self.wB),
                                           ptr(self.paramsB), self.epsilon, env.seed, self.seed_net, env.counter,
                                           steps, ptr(self.heads), ptr(env.obsA), ptr(env.obsB), ctypes_ref(rp),
                                           ptr(self.stats), env.n, stream_ptr()), "pm_rollout_push")
            if steps and env.n:
                if replay.size == 0:
                    replay.max_prio = 1.0
                replay.advance(steps * env.n)
        env.counter += steps
        if not sync:
            return self.stats
        return dict(zip(names, (int(v) for v in self.stats[:len(names)].cpu().tolist())))


def _weights(t, size, name, device):
    require_device(t, name)
    t = t.reshape(-1)
    if t.numel() != size or t.dtype != torch.float32:
        raise ValueError(f"{name} must hold {size} float32 values, got {t.numel()} {t.dtype}")
    t = t.to(device).contiguous()  # the env's device (a no-op when already there)
    if t.data_ptr() % 16:
        t = t.clone()
    return t
