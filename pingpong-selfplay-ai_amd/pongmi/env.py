"""Batched PongEnv2P on the device (K1: pm_env_reset / pm_env_step).

`PongEnv2PBatch` keeps n arenas as struct-of-arrays in HBM: one fp64 slab [7, n] (ball_x, ball_y,
ball_vx, ball_vy, spin, top_paddle_x, bottom_paddle_x) and one int32 slab [4, n] (scoreA, scoreB,
bounce_count, serves). Every call is a single kernel launch on the current stream; nothing
synchronises the host unless the caller reads a result.

Serves (reset draws, envs/my_pong_env_2p.py:94-110) come either from device Philox (production)
or from a host table drawn with CPython's `random` exactly like the reference (parity mode):
`serve_table_from_random`.
"""
import math
import random as _pyrandom

import numpy as np
import torch

from . import _lib
from ._lib import check, ptr, stream_ptr

F64_FIELDS = ("x", "y", "vx", "vy", "spin", "top", "bot")
I32_FIELDS = ("scoreA", "scoreB", "bounces", "serves")

# PongEnv2P.__init__ defaults (envs/my_pong_env_2p.py:19-37)
ENV_DEFAULTS = dict(render_size=400, paddle_width=0.2, paddle_speed=0.02, max_score=3, enable_render=False,
                    enable_spin=True, magnus_factor=0.01, restitution=0.9, friction=0.2, ball_mass=1.0,
                    world_ball_radius=0.03, ball_speed_range=(0.01, 0.05), spin_range=(-10, 10),
                    ball_angle_intervals=None, speed_scale_every=3, speed_increment=0.2)


def env_config(**kw):
    """Resolve PongEnv2P kwargs (unknown keys rejected, like the reference constructor)."""
    unknown = set(kw) - set(ENV_DEFAULTS)
    if unknown:
        raise TypeError(f"PongEnv2P got unexpected keyword arguments {sorted(unknown)}")
    c = dict(ENV_DEFAULTS)
    c.update(kw)
    if not c["ball_angle_intervals"]:
        c["ball_angle_intervals"] = [[-60, -30], [30, 60]]
    return c


def env_params(**kw):
    """pm_env_params from PongEnv2P kwargs. The derived constants are evaluated here with the
    reference's own Python expressions so the device reproduces them bit for bit."""
    c = env_config(**kw)
    if int(c["speed_scale_every"]) <= 0:
        raise ZeroDivisionError("speed_scale_every must be positive (bounce_count % speed_scale_every)")
    p = _lib.EnvParams()
    p.paddle_width = c["paddle_width"]
    p.paddle_speed = c["paddle_speed"]
    p.magnus_factor = c["magnus_factor"]
    p.restitution = c["restitution"]
    p.friction = c["friction"]
    p.ball_mass = c["ball_mass"]
    p.radius = c["world_ball_radius"]
    p.speed_lo, p.speed_hi = c["ball_speed_range"]
    p.spin_lo, p.spin_hi = c["spin_range"]
    (p.ang0_lo, p.ang0_hi), (p.ang1_lo, p.ang1_hi) = c["ball_angle_intervals"][0], c["ball_angle_intervals"][1]
    m, R = c["ball_mass"], c["world_ball_radius"]
    p.half_width = c["paddle_width"] / 2                 # :152,190
    p.speed_scale = 1.0 + c["speed_increment"]           # :230
    p.inertia = (2 / 5) * m * R ** 2                     # envs/physics.py:9
    p.jt_coef = 2 * m / 7.0                              # envs/physics.py:10
    p.inv_mass = 1.0 / m if m else float("inf")          # divisors of physics.py:20-21 (see pongmi.h)
    p.inv_inertia = 1.0 / p.inertia if p.inertia else float("inf")
    p.max_score = int(c["max_score"])
    p.speed_scale_every = int(c["speed_scale_every"])
    p.enable_spin = int(bool(c["enable_spin"]))
    return p


def draw_serve(rng, cfg):
    """One reset() serve from a `random`-module stream, in the reference's draw order and with its
    expressions (envs/my_pong_env_2p.py:94-110). Returns (vx, vy, spin)."""
    speed = rng.uniform(*cfg["ball_speed_range"])
    if rng.random() < 0.5:
        angle_deg = rng.uniform(*cfg["ball_angle_intervals"][0])
    else:
        angle_deg = rng.uniform(*cfg["ball_angle_intervals"][1])
    angle_rad = math.radians(angle_deg)
    return speed * math.cos(angle_rad), speed * math.sin(angle_rad), rng.uniform(*cfg["spin_range"])


def serve_table_from_random(seeds, serves, **env_kw):
    """Parity-mode serve table [n, serves, 3]: arena i draws from random.Random(seeds[i]) the
    serves the reference would draw after random.seed(seeds[i])."""
    cfg = env_config(**env_kw)
    tab = np.zeros((len(seeds), serves, 3), np.float64)
    for i, s in enumerate(seeds):
        rng = _pyrandom.Random(int(s))
        for k in range(serves):
            tab[i, k] = draw_serve(rng, cfg)
    return tab


class PongEnv2PBatch:
    """n independent PongEnv2P arenas advanced in lockstep on one device.

    step(aA, aB) -> ((obsA, obsB), (rA, rB), done, info), all device tensors: obs [n, 7] f32,
    rewards [n] f32, done [n] u8. With autoreset=True finished arenas are served again inside the
    same kernel; obs then holds the post-reset observation and info['term_obsA'/'term_obsB'] the
    observation the step returned before the reset (what the reference pushes to replay as next
    state). autoreset="done" writes the term rows of finished arenas only (the others keep old
    contents: next state = where(done, term_obs, obs)), which saves 56 B of stores per env-step.
    Production (Philox) serves of autoreset arenas are keyed by (arena, self.counter), the number
    of step() calls so far (ABI 15); a parity-mode serve table is indexed by the per-arena serve
    count instead, as pm_env_reset does."""

    def __init__(self, n, device="cuda", seed=0, serve_table=None, autoreset=False, **env_kw):
        self.lib = _lib.load()
        self.n = int(n)
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise _lib.PongmiError("PongEnv2PBatch runs on a ROCm device only (libpongmi has no CPU path)")
        self.cfg = env_config(**env_kw)
        self.params = env_params(**env_kw)
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0  # env steps taken: the Philox key of each step's autoreset serves
        if autoreset not in (False, True, 0, 1, "done"):
            raise ValueError(f"autoreset must be False, True or 'done', got {autoreset!r}")
        self.autoreset = 2 if autoreset == "done" else int(bool(autoreset))
        n, dev = self.n, self.device
        self.f64 = torch.zeros((7, n), dtype=torch.float64, device=dev)
        self.i32 = torch.zeros((4, n), dtype=torch.int32, device=dev)
        self.state = _lib.EnvState(*[ptr(self.f64[k]) for k in range(7)], *[ptr(self.i32[k]) for k in range(4)])
        self.obsA = torch.zeros((n, 7), dtype=torch.float32, device=dev)
        self.obsB = torch.zeros((n, 7), dtype=torch.float32, device=dev)
        self.rA = torch.zeros(n, dtype=torch.float32, device=dev)
        self.rB = torch.zeros(n, dtype=torch.float32, device=dev)
        self.done = torch.zeros(n, dtype=torch.uint8, device=dev)
        self.term_obsA = torch.zeros((n, 7), dtype=torch.float32, device=dev) if autoreset else None
        self.term_obsB = torch.zeros((n, 7), dtype=torch.float32, device=dev) if autoreset else None
        self.set_serve_table(serve_table)

    # ------------------------------------------------------------------ serves
    def set_serve_table(self, table):
        """table: None (Philox serves) or array [n, cap, 3] of (vx, vy, spin)."""
        if table is None:
            self.inject, self.inject_cap = None, 0
            return
        t = torch.as_tensor(np.ascontiguousarray(table, np.float64))
        if t.dim() != 3 or t.shape[0] != self.n or t.shape[2] != 3:
            raise ValueError(f"serve table must be [n={self.n}, cap, 3], got {tuple(t.shape)}")
        self.inject = t.to(self.device)
        self.inject_cap = int(t.shape[1])

    # ------------------------------------------------------------------ API
    def reset(self, mask=None):
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
        check(self.lib.pm_env_reset(ctypes_ref(self.params), ctypes_ref(self.state), ptr(mask), ptr(self.inject),
                                    self.inject_cap, self.seed, ptr(self.obsA), ptr(self.obsB), None, self.n,
                                    stream_ptr()), "pm_env_reset")
        return self.obsA, self.obsB

    def step(self, aA, aB):
        aA = _as_actions(aA, self.n, self.device)
        aB = _as_actions(aB, self.n, self.device)
        check(self.lib.pm_env_step(ctypes_ref(self.params), ctypes_ref(self.state), ptr(aA), ptr(aB), ptr(self.obsA),
                                   ptr(self.obsB), ptr(self.rA), ptr(self.rB), ptr(self.done), ptr(self.term_obsA),
                                   ptr(self.term_obsB), self.autoreset, ptr(self.inject), self.inject_cap,
                                   self.seed, self.counter, None, self.n, stream_ptr()), "pm_env_step")
        self.counter += 1
        info = {}
        if self.autoreset:
            info = {"term_obsA": self.term_obsA, "term_obsB": self.term_obsB}
        return (self.obsA, self.obsB), (self.rA, self.rB), self.done, info

    # ------------------------------------------------------------------ state access
    def get_state(self):
        """Host copy: dict of numpy arrays (fp64 fields and int32 counters)."""
        f = self.f64.cpu().numpy()
        i = self.i32.cpu().numpy()
        out = {k: f[j].copy() for j, k in enumerate(F64_FIELDS)}
        out.update({k: i[j].copy() for j, k in enumerate(I32_FIELDS)})
        return out

    def set_state(self, st):
        f = np.stack([np.asarray(st[k], np.float64) for k in F64_FIELDS])
        i = np.stack([np.asarray(st.get(k, np.zeros(self.n)), np.int32) for k in I32_FIELDS])
        self.f64.copy_(torch.from_numpy(f))
        self.i32.copy_(torch.from_numpy(i))


def _as_actions(a, n, device):
    if not torch.is_tensor(a):
        a = torch.as_tensor(np.asarray(a))
    a = a.to(device=device, dtype=torch.int8).reshape(-1).contiguous()
    if a.numel() != n:
        raise ValueError(f"expected {n} actions, got {a.numel()}")
    return a


def ctypes_ref(s):
    import ctypes
    return ctypes.byref(s)
