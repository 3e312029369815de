"""ctypes binding of libpongmi.so (include/pongmi.h).

The library is the product's only compute path: if it is missing or fails to load, every entry
point raises — there is no CPU or pure-PyTorch fallback for the hot path.

torch must be imported before the library is loaded: both link libamdhip64.so.7, and loading
torch first makes the dynamic loader resolve libpongmi's HIP runtime to the instance torch already
initialised, so device pointers and streams are shared.
"""
import ctypes
import os

import numpy as np

import torch  # noqa: F401  (load order: see module docstring)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PONGMI_LIB", os.path.join(HERE, "libpongmi.so"))

c_double, c_float = ctypes.c_double, ctypes.c_float
c_i32, c_i64, c_u64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64
c_void_p = ctypes.c_void_p

PM_QNET_NP = 5452
PM_QNET_NHEAD = 520
PM_QNET_HEAD_OFF = 4672
PM_QNET_EPS_OFF = 5192
PM_QNET_NW = 9944
PM_GRAD_EPISODES, PM_GRAD_UPDATED, PM_GRAD_LEN = 520, 521, 528
PM_QNET_PLAIN = 4936
PM_RNN_NP = 192012
PM_RNN_NPARAM = 174984
PM_RNN_NW = 157456
PM_TRANS_F = 16
PM_MAX_BATCH = 256
PM_FOLD_EVAL, PM_FOLD_TRAIN, PM_FOLD_TRAIN_FRESH = 0, 1, 2
PM_ACT_ALL, PM_ACT_B, PM_ACT_A = 0, 1, 2
PM_UPD_FIRST, PM_UPD_LAST = 1, 2
PM_COMM_ID_BYTES = 128
ABI_VERSION = 23
PM_TIMER_ACTENV, PM_TIMER_LEARN, PM_TIMER_RNN_ACT, PM_TIMER_ENV_STEP, PM_TIMER_ROLLOUT, PM_TIMER_DRQN = 0, 1, 2, 3, 4, 5
PM_TIMER_LEARN_MULTI, PM_TIMER_N = 6, 7
PM_ROLL_HEADS = 264


class EnvParams(ctypes.Structure):
    _fields_ = [(n, c_double) for n in (
        "paddle_width", "paddle_speed", "magnus_factor", "restitution", "friction", "ball_mass", "radius",
        "speed_lo", "speed_hi", "spin_lo", "spin_hi", "ang0_lo", "ang0_hi", "ang1_lo", "ang1_hi",
        "half_width", "speed_scale", "inertia", "jt_coef", "inv_mass", "inv_inertia")] + \
        [("max_score", c_i32), ("speed_scale_every", c_i32), ("enable_spin", c_i32), ("_pad", c_i32)]


class EnvState(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("x", "y", "vx", "vy", "spin", "top", "bot",
                                        "scoreA", "scoreB", "bounces", "serves")]


class Ctrl(ctypes.Structure):
    _fields_ = [("step", c_u64), ("pos", c_i64), ("size", c_i64), ("train_steps", c_i64), ("frame_idx", c_i64),
                ("episodes", c_i64), ("epsilon", c_double), ("max_prio", c_float), ("last_loss", c_float),
                ("ep_step", c_i64), ("win_A", c_i64), ("ep_A", c_i64), ("win_P", c_i64), ("ep_P", c_i64),
                ("reward_B", c_double), ("status", c_i32), ("max_bits", c_i32)]


class SelfPlay(ctypes.Structure):
    _fields_ = [("env", EnvParams), ("st", EnvState)] + \
        [(n, c_void_p) for n in ("opp", "ep_reward", "w_opp", "paramsB", "paramsT", "w_B", "adam_m", "adam_v",
                                 "trans", "prios", "per_work", "idx", "isw", "grad", "partials", "obsA", "obsB", "aA",
                                 "aB", "hfeat", "learn_heads", "ctrl", "opp_list", "opp_cnt")] + \
        [("n", c_i32), ("n_pool", c_i32), ("batch", c_i32), ("world", c_i32), ("chunk_A", c_i32), ("chunk_P", c_i32),
         ("fuse_apply", c_i32), ("_pad0", c_i32), ("cap", c_i64)] + \
        [(n, c_double) for n in ("gamma", "alpha", "lr", "beta1", "beta2", "adam_eps", "min_epsilon", "epsilon_decay",
                                 "pool_ratio", "beta_start")] + \
        [("beta_frames", c_i64), ("target_update_interval", c_i64), ("seed_env", c_u64), ("seed_net", c_u64),
         ("featB", c_void_p), ("frow", c_void_p), ("frow_ready", c_i32), ("_pad1", c_i32)]


class RollReplay(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("trans", "prios", "per_work", "ep_reward")] + \
        [("pos", c_i64), ("cap", c_i64), ("prio", c_float), ("alpha", c_float)]


class DrqnStats(ctypes.Structure):
    _fields_ = [("steps", c_i64), ("adam_t", c_i64), ("loss", c_float), ("norm", c_float), ("q_mean", c_float),
                ("status", c_i32)]


class Drqn(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("params", "target", "adam_m", "adam_v", "grad", "work", "stats", "obs", "next",
                                        "act", "rew", "done", "enable")] + \
        [("batch", c_i32), ("T", c_i32), ("target_update_interval", c_i64)] + \
        [(n, c_double) for n in ("gamma", "lr", "beta1", "beta2", "adam_eps", "max_norm")] + \
        [("poll_limit", c_i32), ("reserved", c_i32)]


class RnnCtrl(ctypes.Structure):
    _fields_ = [("step", c_u64), ("episodes", c_i64), ("seq_count", c_i64), ("seq_size", c_i64), ("epsilon", c_double),
                ("win_A", c_i64), ("ep_A", c_i64), ("win_P", c_i64), ("ep_P", c_i64), ("reward_B", c_double),
                ("status", c_i32), ("train", c_i32)]


class RnnSelfPlay(ctypes.Structure):
    _fields_ = [("env", EnvParams), ("st", EnvState)] + \
        [(n, c_void_p) for n in ("opp", "ep_reward", "ep_len", "ep_steps", "reset", "w_opp", "paramsB", "w_B", "hA",
                                 "cA", "hB", "cB", "obsA", "obsB", "aA", "aB", "trans", "seq_eps", "seq_mark", "fin",
                                 "partials", "opp_list", "opp_cnt", "enable", "ctrl")] + \
        [(n, c_i32) for n in ("n", "n_pool", "depth", "T", "chunk_A", "chunk_P", "max_steps", "_pad")] + \
        [("seq_cap", c_i64), ("min_episodes", c_i64)] + \
        [(n, c_double) for n in ("min_epsilon", "epsilon_decay", "pool_ratio")] + \
        [("seed_env", c_u64), ("seed_net", c_u64), ("hA_in", c_void_p), ("cA_in", c_void_p), ("qA", c_void_p),
         ("qB", c_void_p)]


CTRL_DTYPE_BYTES = ctypes.sizeof(Ctrl)

# name -> (restype, argtypes)
_SIGS = {
    "pm_env_reset": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_u64, c_void_p, c_void_p, c_void_p, c_i32,
                             c_void_p]),
    "pm_env_step": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_i32, c_void_p, c_i32, c_u64, c_u64, c_void_p, c_i32, c_void_p]),
    "pm_collide": (c_i32, [c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_env_step1": (c_i32, [c_void_p, c_void_p, c_i32, c_i32, c_void_p, ctypes.c_uint32, c_void_p]),
    "pm_env_reset1": (c_i32, [c_void_p, c_double, c_double, c_double, c_void_p, ctypes.c_uint32, c_void_p]),
    "pm_collide1": (c_i32, [c_void_p, c_double, c_void_p, ctypes.c_uint32, c_void_p]),
    "pm_host_mapped_alloc": (c_void_p, [ctypes.c_int64, ctypes.POINTER(c_void_p)]),
    "pm_host_mapped_free": (c_i32, [c_void_p]),
    "pm_qnet_fold": (c_i32, [c_void_p, c_void_p, c_i32, c_u64, c_u64, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_qnet_q": (c_i32, [c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_qnet_act": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_u64, c_u64,
                            c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_i32, c_i32, c_void_p]),
    "pm_rnn_fold": (c_i32, [c_void_p, c_void_p, c_i32, c_u64, c_u64, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_rnn_q": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_rnn_act": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_float, c_void_p, c_u64, c_u64, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_i32, c_i32, c_i32, c_void_p, c_void_p, c_void_p]),
    "pm_play": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_void_p, c_void_p, c_i32, c_i32,
                        c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "pm_rollout": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_u64, c_u64, c_u64, c_i32,
                           c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_per_build": (c_i32, [c_void_p, c_i64, c_float, c_void_p, c_void_p]),
    "pm_rollout_push": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_u64, c_u64, c_u64,
                                c_i32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_drqn_work_bytes": (c_i64, [c_i32, c_i32]),
    "pm_drqn_init": (c_i32, [c_void_p, c_void_p]),
    "pm_drqn_grads": (c_i32, [c_void_p, c_void_p]),
    "pm_drqn_apply": (c_i32, [c_void_p, c_void_p]),
    "pm_drqn_update": (c_i32, [c_void_p, c_void_p]),
    "pm_rnn_selfplay_init": (c_i32, [c_void_p, c_void_p]),
    "pm_rnn_selfplay_act": (c_i32, [c_void_p, c_void_p]),
    "pm_rnn_selfplay_env": (c_i32, [c_void_p, c_void_p, c_void_p]),
    "pm_rnn_selfplay_rollout": (c_i32, [c_void_p, c_void_p, c_void_p]),
    "pm_rnn_selfplay_step": (c_i32, [c_void_p, c_void_p, c_void_p]),
    "pm_rnn_selfplay_sample": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_rnn_selfplay_step_multi": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_per_work_bytes": (c_i64, [c_i64]),
    "pm_per_sample": (c_i32, [c_void_p, c_i64, c_float, c_float, c_void_p, c_u64, c_u64, c_void_p, c_void_p, c_i32,
                              c_void_p, c_void_p]),
    "pm_per_update": (c_i32, [c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_selfplay_init": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_prepare": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_repair_tree": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_rollout": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_act": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_env": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_learn": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_apply": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_step": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_act_part": (c_i32, [c_void_p, c_i32, c_void_p]),
    "pm_selfplay_learn_act": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_actenv": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_step_overlap": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_learn_ex": (c_i32, [c_void_p, c_i32, c_i32, c_void_p]),
    "pm_selfplay_apply_ex": (c_i32, [c_void_p, c_i32, c_void_p]),
    "pm_selfplay_resample": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_commit": (c_i32, [c_void_p, c_void_p]),
    "pm_selfplay_step_multi": (c_i32, [c_void_p, c_i32, c_void_p]),
    "pm_rnn_selfplay_act_part": (c_i32, [c_void_p, c_i32, c_void_p]),
    "pm_rnn_selfplay_step_overlap": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p]),
    "pm_rnn_selfplay_finish_overlap": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p, c_void_p]),
    "pm_comm_unique_id": (c_i32, [ctypes.c_char_p, c_void_p]),
    "pm_comm_init": (c_i32, [ctypes.c_char_p, c_void_p, c_i32, c_i32, ctypes.POINTER(c_void_p)]),
    "pm_comm_allreduce_f32": (c_i32, [c_void_p, c_void_p, c_i64, c_void_p]),
    "pm_comm_destroy": (c_i32, [c_void_p]),
    "pm_comm_info": (c_i32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "pm_selfplay_step_sharded": (c_i32, [c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_rnn_selfplay_step_sharded": (c_i32, [c_void_p, c_void_p, c_void_p, c_i32, c_void_p]),
    "pm_rnn_selfplay_step_sharded_overlap": (c_i32, [c_void_p, c_void_p, c_void_p, c_i32, c_void_p, c_void_p]),
    "pm_timer_arm": (c_i32, [c_i32]),
    "pm_timer_read": (c_i32, [c_i32, ctypes.POINTER(c_float)]),
    "pm_last_error": (ctypes.c_char_p, []),
    "pm_abi_version": (c_i32, []),
    "pm_sizeof": (c_i32, [c_i32]),
}
EXPORTED = tuple(_SIGS)

_lib = None


class PongmiError(RuntimeError):
    pass


def load():
    """Load libpongmi.so once; raise (never fall back) if it is absent or inconsistent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise PongmiError(f"libpongmi.so not found at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (or `make -C pingpong-selfplay-ai_amd/csrc`) first")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    if L.pm_abi_version() != ABI_VERSION:
        raise PongmiError(f"libpongmi ABI {L.pm_abi_version()} != {ABI_VERSION}")
    for which, cls in ((0, EnvParams), (1, EnvState), (2, Ctrl), (3, SelfPlay), (4, Drqn), (5, DrqnStats), (6, RnnCtrl),
                       (7, RnnSelfPlay)):
        if L.pm_sizeof(which) != ctypes.sizeof(cls):
            raise PongmiError(f"struct layout mismatch for {cls.__name__}: C {L.pm_sizeof(which)} "
                              f"vs ctypes {ctypes.sizeof(cls)}")
    _lib = L
    return L


def timer_arm(kernel):
    """Queue one launch of `kernel` (PM_TIMER_*) to record its own begin/end (pm_timer_arm)."""
    check(load().pm_timer_arm(int(kernel)), "pm_timer_arm")


def timer_read(kernel):
    """Duration in seconds of the oldest unread timed launch of `kernel` (waits for it)."""
    ms = c_float()
    check(load().pm_timer_read(int(kernel), ctypes.byref(ms)), "pm_timer_read")
    return ms.value * 1e-3


class MappedSlot:
    """A small host-mapped buffer (pm_host_mapped_alloc) for the scalar drop-ins' one-launch calls:
    the kernel writes its results and then a sequence number into the word after them; wait()
    polls that word (bounded: after `timeout` s it synchronises the stream and raises)."""

    def __init__(self, nwords, seq_word):
        self.lib = load()
        dev = c_void_p()
        self.host = self.lib.pm_host_mapped_alloc(4 * int(nwords), ctypes.byref(dev))
        if not self.host:
            raise PongmiError("pm_host_mapped_alloc failed")
        self.dev = dev.value
        self.words = (ctypes.c_uint32 * int(nwords)).from_address(self.host)
        # float32 / float64 views of the same words, made once (a per-call from_address + frombuffer
        # costs a few microseconds of the ~10-us scalar step)
        self.f32 = np.ctypeslib.as_array((ctypes.c_float * int(nwords)).from_address(self.host))
        self.f64 = np.ctypeslib.as_array((ctypes.c_double * (int(nwords) // 2)).from_address(self.host))
        self.seq_word = int(seq_word)
        self.seq = 0

    def next_seq(self):
        self.seq = (self.seq + 1) & 0xFFFFFFFF or 1
        return self.seq

    def wait(self, timeout=5.0):
        w, k, want = self.words, self.seq_word, self.seq
        for _ in range(2000):
            if w[k] == want:
                return
        import time
        t0 = time.perf_counter()
        while w[k] != want:
            if time.perf_counter() - t0 > timeout:
                import torch
                torch.cuda.synchronize()
                if w[k] != want:
                    raise PongmiError("scalar drop-in: the device never published its result")
                return

    def floats(self, lo, hi):
        return self.f32[lo:hi].copy()

    def doubles(self, lo, hi):
        return self.f64[lo:hi].copy()

    def __del__(self):
        try:
            if self.host:
                self.lib.pm_host_mapped_free(self.host)
                self.host = None
        except Exception:
            pass


def check(rc, what=""):
    if rc != 0:
        msg = load().pm_last_error().decode(errors="replace")
        raise PongmiError(f"{what or 'libpongmi'} failed (rc={rc}): {msg}")


def ptr(t):
    """Device (or host) address of a tensor, None for None."""
    if t is None:
        return None
    return t.data_ptr()


def stream_ptr(stream=None):
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def current_stream():
    """The current torch stream object (callers that cache its handle keep the object alive)."""
    return torch.cuda.current_stream()


def require_device(t, name):
    if not t.is_cuda:
        raise PongmiError(f"{name} must be a ROCm device tensor (libpongmi has no CPU path)")
    if not t.is_contiguous():
        raise PongmiError(f"{name} must be contiguous")
