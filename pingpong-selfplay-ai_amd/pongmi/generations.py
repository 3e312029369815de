"""Generation controllers: the promotion / retry / fault logic and checkpoint I/O of
scripts/train_iterative.py (:77-297) and scripts/train_rnn_iterative.py (:225-885) over the batched
learners (SelfPlayLearner, RNNSelfPlayLearner) and evaluators.

Each training try plays until `episodes_per_generation` more episodes have finished across the
arenas (counted on the device, read every `check_every` vector steps; the reference plays exactly
that many episodes one after another).

Replay ratio. The reference trains once per env step (train_iterative.py:243-244,
train_rnn_iterative.py:776-777): one update per pushed transition, ~episodes x mean length
(~38 steps) updates per try, which is what lets its double-DQN target sync every 1000 / 2000
updates within a generation. A vector step pushes n transitions, so the controllers run
U = round(replay_ratio * n) updates per vector step (replay_ratio = 1.0: the reference's ratio) on
a few hundred arenas by default (QNet 512, QNetRNN 64) rather than the bench's 65 536: a try then
costs ~episodes x 38 updates, as the reference's does, and finishes in seconds on the device.

After a try, modelB is evaluated against modelA and the pool with the batched evaluators (serves
and pool draws from the global `random` stream, as the reference), and promoted, retried or saved
as a fault exactly as the reference decides. Checkpoints are the
reference's dicts (same keys, same order, state_dicts with the reference's key names and an Adam
state_dict), written with torch.save and loadable by the reference's scripts and tests/arena.py.
Console lines keep the reference's formats (win rates in the interval lines are over the episodes
finished since the previous line, the reference's deque holds the last win_rate_interval).
"""
import copy
import os
import time

import torch

from . import _lib, checkpoint
from .evaluate import eval_vs_model, eval_vs_pool
from .tournament import play_matches


def _env_kw(cfg):
    return {k: v for k, v in cfg["env"].items() if k not in ("render_size", "enable_render")}


class _Progress:
    """Interval console lines + the episode budget of one try."""

    def __init__(self, L, interval, fmt, log):
        self.L, self.interval, self.fmt, self.log = L, int(interval), fmt, log
        self.start = self.t0 = time.time()
        c = L.counters()
        self.last = c
        self.next_mark = (c["episodes"] // self.interval + 1) * self.interval

    def tick(self, c):
        if c["episodes"] < self.next_mark:
            return
        now = time.time()
        d = {k: c[k] - self.last[k] for k in ("win_A", "ep_A", "win_P", "ep_P")}
        avgA = d["win_A"] / d["ep_A"] if d["ep_A"] else (-1.0 if self.fmt == "rnn" else 0.0)
        avgP = d["win_P"] / d["ep_P"] if d["ep_P"] else (-1.0 if self.fmt == "rnn" else 0.0)
        n = c["episodes"] // self.interval * self.interval
        if self.fmt == "rnn":
            self.log(f"[Ep {n}] WinRate (vs A):{avgA:.2f} (vs P):{avgP:.2f} | Eps: {c['epsilon']:.3f} | "
                     f"Last Reward B: {c.get('reward_B', 0.0):.1f} | Interval:{now - self.t0:.1f}s | Total:{(now - self.start) / 60:.1f}min")
        else:
            self.log(f"[Ep {n}] vs A:{avgA:.2f}, vs Pool:{avgP:.2f}, interval:{now - self.t0:.1f}s, "
                     f"total:{(now - self.start) / 60:.1f}min")
        self.t0, self.last = now, c
        self.next_mark = (c["episodes"] // self.interval + 1) * self.interval


def updates_for(n_arenas, replay_ratio=1.0, updates_per_step=None):
    """Updates per vector step: explicit, or replay_ratio updates per pushed transition."""
    if updates_per_step is not None:
        return max(1, int(updates_per_step))
    return max(1, int(round(float(replay_ratio) * int(n_arenas))))


def _play_episodes(L, episodes, progress, check_every, on_check=None, step=None):
    e0 = L.counters()["episodes"]
    step = step or L.step
    while True:
        for _ in range(check_every):
            step()
        c = L.counters()
        if hasattr(L, "repair_tree") and L.repair_tree(c):  # a tree-refresh timeout: rebuild the stale sums
            c = L.counters()
        progress.tick(c)
        if on_check:
            on_check(c)
        if c["episodes"] - e0 >= episodes:
            return c


# ---------------------------------------------------------------------------------------- QNet
class QNetGenerations:
    """scripts/train_iterative.py: generations of modelB (NoisyNet heads, PER double DQN) against a
    frozen modelA and a pool read once from the init checkpoint's directory."""

    def __init__(self, cfg, n_arenas=512, device="cuda", seed=0, log=print, check_every=4, replay_ratio=1.0,
                 updates_per_step=None):
        from models.qnet import QNet
        from .selfplay import SelfPlayLearner
        t = cfg["training"]
        self.cfg, self.t, self.log, self.check_every = cfg, t, log, int(check_every)
        self.env_kw = _env_kw(cfg)
        self.ckpt_dir = os.path.dirname(t["init_model_path"]) or "."
        base_cp = checkpoint.load(t["init_model_path"])
        old = base_cp.get("modelB", base_cp.get("model"))
        net = QNet(7, 3)
        net.load_state_dict(old, strict=False)  # strict=False (:89-94): keys it lacks keep their init
        self.old_state = copy.deepcopy(net.state_dict())
        epsilon = base_cp.get("epsilon", t["min_epsilon"])
        episode = base_cp.get("episode", 0)
        log(f"[INFO] Loaded init_model from {t['init_model_path']}, eps={epsilon}, episode={episode}")
        pool = []
        for fn in os.listdir(self.ckpt_dir):  # :199-207
            if not fn.endswith(".pth"):
                continue
            cp2 = checkpoint.load(os.path.join(self.ckpt_dir, fn))
            st2 = cp2.get("modelB", cp2.get("model", None))
            if st2 is None:
                continue
            m = QNet(7, 3)
            m.load_state_dict(st2, strict=False)
            pool.append(copy.deepcopy(m.state_dict()))
        self.pool = pool
        log(f"[INFO] Loaded {len(pool)} pool models.")
        self.L = SelfPlayLearner(self.env_kw, n_arenas, self.old_state, self.old_state, pool,
                                 batch=t["batch_size"], memory_size=t["memory_size"], gamma=t["gamma"], lr=t["lr"],
                                 epsilon=epsilon, min_epsilon=t["min_epsilon"], epsilon_decay=t["epsilon_decay"],
                                 target_update_interval=t["target_update_interval"],
                                 pool_ratio=t["opponent_pool_ratio"], episode=episode, seed=seed, device=device,
                                 updates_per_step=updates_for(n_arenas, replay_ratio, updates_per_step))
        self.done_generations = 0
        self.current_generation = 0

    def _save(self, fn):
        L = self.L
        c = L.counters()
        torch.save({"modelB": checkpoint.cpu_state(L.modelB_state_dict()), "optimizer": L.optimizer_state_dict(),
                    "epsilon": c["epsilon"], "episode": c["episodes"],
                    "modelA": checkpoint.cpu_state(L.modelA_state_dict())}, os.path.join(self.ckpt_dir, fn))

    def evaluate(self, rng=None):
        """(win vs modelA, win vs pool): eval_vs_model / eval_vs_pool (:171-196) with modelA and modelB
        as the reference has them (train mode, their current epsilon buffers), pool nets in eval mode."""
        L, E = self.L, int(self.t["eval_episodes"])
        B = (L.modelB_state_dict(), _lib.PM_FOLD_TRAIN)
        A = (L.modelA_state_dict(), _lib.PM_FOLD_TRAIN if L.modelA_noisy else _lib.PM_FOLD_EVAL)
        wA = eval_vs_model(self.env_kw, A, B, E, rng=rng)
        wP = eval_vs_pool(self.env_kw, B, [(sd, _lib.PM_FOLD_EVAL) for sd in self.pool], E, rng=rng)
        return wA, wP

    def run(self, rng=None):
        t, L, log = self.t, self.L, self.log
        while self.done_generations < t["max_generations"]:
            self.current_generation += 1
            g = self.current_generation
            log(f"\n=== Generation {g} ===")
            tries = 0
            while True:
                tries += 1
                log(f"  [Gen {g}] try {tries}/{t['max_retries_for_generation']}")
                _play_episodes(L, t["episodes_per_generation"], _Progress(L, t["win_rate_interval"], "qnet", log),
                               self.check_every)
                wA, wP = self.evaluate(rng)
                c = L.counters()
                L.check_status(c)
                log(f"[Gen {g}] vs A:{wA:.2f}, vs Pool:{wP:.2f}, eps={c['epsilon']:.3f}")
                if wA >= t["curr_win_threshold"] and wP >= t["pool_win_threshold"]:
                    log(f"升級! generation {g} done.")
                    L.set_modelA(L.modelB_state_dict())
                    fn = f"model{t['model_id']}-{g}.pth"
                    self._save(fn)
                    log(f"[Saved] {fn}")
                    self.done_generations += 1
                    break
                if tries >= t["max_retries_for_generation"]:
                    fn = f"model{t['model_id']}-{g}_fault.pth"
                    self._save(fn)
                    log(f"[Fault] {fn}")
                    L.reset_B(self.old_state)  # reset_B (:213-224)
                    self.done_generations += 1
                    break
                log("未達标，继续尝试…")


# ---------------------------------------------------------------------------------------- QNetRNN
class RNNGenerations:
    """scripts/train_rnn_iterative.py: generations of a QNetRNN modelB (DRQN on sequences) with resume
    from the latest-state checkpoint, per-generation restart of B from A, and promoted models joining
    the runtime pool."""

    def __init__(self, cfg, n_arenas=64, device="cuda", seed=0, log=print, check_every=4, replay_ratio=1.0,
                 updates_per_step=None):
        from models.qnet_rnn import QNetRNN
        from .rnn_selfplay import RNNSelfPlayLearner
        t = cfg["training"]
        g = lambda k, d=None: t.get(k, d)  # noqa: E731  get_cfg (:36-37)
        self.cfg, self.t, self.log, self.check_every = cfg, t, log, int(check_every)
        self.env_kw = _env_kw(cfg)
        self.prefix = g("model_id_prefix", "rnn_agent_2_")
        self.ckpt_dir = g("ckpt_dir_rnn", "checkpoints_rnn")
        os.makedirs(self.ckpt_dir, exist_ok=True)
        self.latest = os.path.join(self.ckpt_dir, g("latest_checkpoint_filename", "latest_rnn_training_state.pth"))
        self.save_every = int(g("save_latest_checkpoint_interval_steps", 10000))
        self.arch = dict(feature_dim=g("feature_dim", 128), lstm_hidden_dim=g("lstm_hidden_dim", 128),
                         lstm_layers=g("lstm_layers", 1), head_hidden_dim=g("head_hidden_dim", 128))
        new = lambda: QNetRNN(7, 3, **self.arch)  # noqa: E731
        init = g("init_model_path_rnn", None)
        sdA = sdB = opt = None
        epsilon, episodes, train_steps, self.old_state = 1.0, 0, 0, None
        resumed = False
        if os.path.exists(self.latest) and self.save_every > 0:  # :231-267
            log(f"[INFO] Loading training state from latest checkpoint: {self.latest}")
            try:
                cp = checkpoint.load(self.latest)
                a, b = new(), new()
                a.load_state_dict(cp["modelA_state"])
                b.load_state_dict(cp["modelB_state"])
                sdA, sdB, opt = a.state_dict(), b.state_dict(), cp["optimizer_B_state"]
                epsilon, episodes = cp["epsilon"], cp["global_episode_count"]
                train_steps = cp["train_steps_count"]
                self.old_state = cp.get("old_state_for_reset") or copy.deepcopy(sdA)
                log(f"[INFO] Resumed from latest checkpoint. Gen to start: {cp['current_generation_active']}, "
                    f"Done Gens: {cp['done_generations_count']}, Eps: {epsilon:.4f}, Global Episodes: {episodes}, "
                    f"Train Steps: {train_steps}")
                resumed = True
            except Exception as e:
                log(f"[ERROR] Failed to load from latest checkpoint {self.latest}: {e}. Will proceed with other "
                    f"init methods.")
                sdA = sdB = opt = None
                epsilon, episodes, train_steps = 1.0, 0, 0
        if not resumed and init and os.path.exists(init):  # :276-318
            log(f"[INFO] Loading initial RNN model from {init}")
            try:
                cp = checkpoint.load(init)
                stA = cp.get("modelA_state", cp.get("modelB_state", cp.get("model")))
                stB = cp.get("modelB_state", stA)
                a, b = new(), new()
                if stA:
                    a.load_state_dict(stA)
                if stB:
                    b.load_state_dict(stB)
                elif stA:
                    b.load_state_dict(stA)
                sdA, sdB = a.state_dict(), b.state_dict()
                self.old_state = cp.get("old_state_for_reset", copy.deepcopy(sdA))
                epsilon, episodes = cp.get("epsilon", 1.0), cp.get("episode", 0)
                train_steps = cp.get("train_steps_count", 0)
                opt = cp.get("optimizer_B_state")
                log(f"[INFO] Initialized from {init}. Epsilon: {epsilon:.4f}")
            except Exception as e:
                log(f"[ERROR] Failed to load from init_model_path {init}: {e}.")
                sdA = sdB = opt = None
                epsilon, episodes, train_steps = 1.0, 0, 0
        if sdA is None or sdB is None:  # :322-339
            log("[INFO] Initializing new RNN models randomly (or due to previous load failure).")
            a = new()
            sdA = sdB = a.state_dict()
            self.old_state = copy.deepcopy(sdA)
            epsilon, episodes, train_steps = 1.0, 0, 0
        pool = []
        for fn in os.listdir(self.ckpt_dir):  # :608-621 (RNN opponents; fault checkpoints skipped)
            if not fn.endswith(".pth") or "fault" in fn:
                continue
            try:
                cp = checkpoint.load(os.path.join(self.ckpt_dir, fn))
                st = cp.get("modelB_state", cp.get("modelA_state", cp.get("model")))
                if st is None:
                    continue
                m = new()
                m.load_state_dict(st)
                pool.append(m.state_dict())
                log(f"[INFO] Loaded RNN pool model: {fn}")
            except Exception as e:
                log(f"Warning: Could not load RNN pool model {fn}: {e}")
        if not pool:
            log("[WARNING] Opponent pool is empty! ModelB will only train against ModelA.")
        self.pool = pool
        self.L = RNNSelfPlayLearner(self.env_kw, n_arenas, sdB, sdA, pool, batch=t["batch_size"],
                                    trace_length=g("trace_length", 8), memory_size=t["memory_size"],
                                    min_episodes_for_training_start=g("min_episodes_for_training_start", 5),
                                    gamma=t["gamma"], lr=t["lr"], epsilon=epsilon, min_epsilon=t["min_epsilon"],
                                    epsilon_decay=t["epsilon_decay"],
                                    target_update_interval=t["target_update_interval"],
                                    pool_ratio=t["opponent_pool_ratio"] or 0.0, grad_clip_norm=g("grad_clip_norm", 1.0),
                                    episode=episodes, seed=seed, device=device,
                                    updates_per_step=updates_for(n_arenas, replay_ratio, updates_per_step),
                                    max_episode_steps=cfg["env"].get("max_episode_steps", 1000))
        if opt:
            self.L.learner.load_optimizer_state_dict(opt)
        self.L.learner.set_train_steps(train_steps)
        # the main loop starts from generation 0 whatever was resumed (:625-626)
        self.done_generations = 0
        self.current_generation = 0
        self._next_save = None
        self._sync_save_mark(train_steps)

    def _sync_save_mark(self, train_steps):
        """Next latest-state save: after update number k * interval (k*interval > train_steps)."""
        self._steps_hi = int(train_steps)  # upper bound of train steps since the last host read
        self._next_save = ((self._steps_hi // self.save_every + 1) * self.save_every if self.save_every > 0
                           else None)

    # ------------------------------------------------------------------ checkpoints
    def _base(self):
        L = self.L
        c = L.counters()
        return L, c, {"modelA_state": checkpoint.cpu_state(L.modelA_state_dict()),
                      "modelB_state": checkpoint.cpu_state(L.modelB_state_dict()),
                      "optimizer_B_state": L.learner.optimizer_state_dict()}

    def save_latest(self, train_steps=None):
        """save_latest_training_checkpoint (:630-667). train_steps: the count to record (default: the
        current one)."""
        L, c, d = self._base()
        ts = c["train_steps"] if train_steps is None else int(train_steps)
        torch.save({**d, "epsilon": c["epsilon"], "global_episode_count": c["episodes"],
                    "current_generation_active": self.current_generation,
                    "done_generations_count": self.done_generations, "train_steps_count": ts,
                    "old_state_for_reset": checkpoint.cpu_state(self.old_state)}, self.latest)

    def _step(self):
        """One vector step. The reference saves the latest state right after the optimizer step of
        update number k * interval, recording train_steps_count = k * interval - 1 (the count before
        that update's increment, :519-528). When update k * interval may fall inside this vector
        step's U updates, the step runs its updates in runs that end exactly there (one host read of
        the train-step count and the enable flag after the rollout: every update of a vector step
        trains or none does) and saves between them; otherwise it is one fused device sequence."""
        L = self.L
        U = L.updates_per_step
        if self._next_save is None or self._steps_hi + U < self._next_save:
            L.step()
            self._steps_hi += U
            return
        L.rollout()
        st = L.learner.stats()["steps"]
        enabled = bool(L.enable.item())
        u = 0
        while u < U:
            run = min(U - u, self._next_save - st) if enabled else U - u
            for _ in range(run):
                if u:
                    L.sample(u)
                L.learner.update()
                u += 1
            if enabled:
                st += run
                if st == self._next_save:
                    self.save_latest(train_steps=st - 1)
                    self._sync_save_mark(st)
        self._steps_hi = st

    def _on_check(self, c):
        self.L.check_status(c, self.log)
        self._steps_hi = int(c["train_steps"])

    def _save_success(self, fn):
        L, c, d = self._base()
        torch.save({**d, "epsilon": c["epsilon"], "episode": c["episodes"], "generation": self.current_generation,
                    "train_steps_count": c["train_steps"],
                    "old_state_for_reset": checkpoint.cpu_state(self.old_state)}, os.path.join(self.ckpt_dir, fn))

    def _save_fault(self, fn):
        L, c, d = self._base()
        torch.save({"modelB_state": d["modelB_state"], "optimizer_B_state": d["optimizer_B_state"],
                    "epsilon": c["epsilon"], "episode": c["episodes"], "generation": self.current_generation,
                    "modelA_state": d["modelA_state"], "train_steps_count": c["train_steps"],
                    "old_state_for_reset": checkpoint.cpu_state(self.old_state)}, os.path.join(self.ckpt_dir, fn))

    # ------------------------------------------------------------------ evaluation
    def evaluate(self, rng=None):
        """eval_model_vs_opponent (:535-587): modelB (eval mode) as player B against modelA, then
        eval_episodes // len(pool) episodes against each pool net (:808-822); a win is B's reward sum
        above A's = the final score. The reference first plays eval_episodes against a uniformly random
        opponent and overwrites that result (:804); that pass only moves the random stream and is
        not played here."""
        from models.qnet_rnn import QNetRNN
        L, E = self.L, int(self.t["eval_episodes"])

        def net(sd):
            m = QNetRNN(7, 3, **self.arch)
            m.load_state_dict(sd)
            return m.eval()

        B = net(L.modelB_state_dict())
        res = play_matches(self.env_kw, {"A": (net(L.modelA_state_dict()), "QNetRNN"), "B": (B, "QNetRNN")},
                           [("A", "B", E)], rng=rng)
        wA = sum(sB > sA for _, _, sA, sB in res) / E
        if not self.pool:
            return wA, 1.0
        each = max(1, E // len(self.pool))
        models = {f"P{k}": (net(sd), "QNetRNN") for k, sd in enumerate(self.pool)}
        models["B"] = (B, "QNetRNN")
        res = play_matches(self.env_kw, models, [(f"P{k}", "B", each) for k in range(len(self.pool))], rng=rng)
        wP = sum(sB > sA for _, _, sA, sB in res) / (len(self.pool) * each)
        return wA, wP

    # ------------------------------------------------------------------ the loop
    def run(self, rng=None):
        t, L, log = self.t, self.L, self.log
        g = lambda k, d=None: t.get(k, d)  # noqa: E731
        max_retries = t["max_retries_for_generation"]
        while self.done_generations < t["max_generations"]:
            self.current_generation += 1
            gen = self.current_generation
            log(f"\n=== RNN Training: Generation {gen}/{t['max_generations']} ===")
            if gen > 1:  # B restarts from A with a new optimizer and exploration (:711-722)
                eps = g("initial_epsilon_per_generation", 1.0)
                L.reset_B(L.modelA_state_dict(), epsilon=eps, reset_train_steps=False)
                log(f"[INFO] New generation: modelB starts from modelA's state. Epsilon reset to {eps}.")
            success = False
            for i_try in range(1, max_retries + 1):
                log(f"  [Gen {gen}] Attempt {i_try}/{max_retries}")
                _play_episodes(L, t["episodes_per_generation"], _Progress(L, t["win_rate_interval"], "rnn", log),
                               self.check_every, self._on_check, self._step)
                log(f"  [Gen {gen}, Try {i_try}] Evaluating modelB...")
                wA, wP = self.evaluate(rng)
                c = L.counters()
                log(f"  [Gen {gen}, Try {i_try}] Eval Results: vs A:{wA:.2f}, vs Pool:{wP:.2f}, Eps:{c['epsilon']:.3f}")
                if wA >= t["curr_win_threshold"] and wP >= t["pool_win_threshold"]:
                    log(f"  SUCCESS! ModelB passed thresholds in Gen {gen}, Try {i_try}.")
                    L.set_modelA(L.modelB_state_dict())
                    self.old_state = copy.deepcopy(L.modelA_state_dict())
                    fn = f"{self.prefix}{gen}.pth"
                    self._save_success(fn)
                    log(f"  [Saved] Checkpoint: {os.path.join(self.ckpt_dir, fn)}")
                    self.pool.append(L.modelA_state_dict())
                    L.add_pool_model(self.pool[-1])
                    log(f"  Added {fn} to the runtime opponent pool (now {len(self.pool)} models).")
                    self.done_generations += 1
                    success = True
                    break
                log(f"  ModelB did not meet thresholds in Gen {gen}, Try {i_try}. Continuing...")
            if not success:
                log(f"  FAILURE! ModelB FAILED to pass thresholds after {max_retries} tries in Gen {gen}.")
                fn = f"{self.prefix}{gen}_fault.pth"
                self._save_fault(fn)
                log(f"  [Fault Saved] Checkpoint: {os.path.join(self.ckpt_dir, fn)}")
                self._reset_b_for_new_attempt()
                self.done_generations += 1

    def _reset_b_for_new_attempt(self):
        """reset_model_b_for_new_attempt (:669-702): B from the init checkpoint's modelB_state when it
        has one, else from modelA; new optimizer, epsilon 1.0, train_steps_count 0."""
        self.log("[INFO] Resetting modelB for a new attempt in current generation.")
        init = self.t.get("init_model_path_rnn", None)
        state = None
        if init and os.path.exists(init):
            cp = checkpoint.load(init)
            if "modelB_state" in cp:
                state = cp.get("modelB_state", cp.get("model"))
                self.log("[INFO] modelB reset to state from init_model_path.")
        if state is None:
            state = self.L.modelA_state_dict()
            self.log("[INFO] modelB reset to current modelA's state.")
        self.L.reset_B(state, epsilon=1.0, reset_train_steps=True)
        self._sync_save_mark(0)
