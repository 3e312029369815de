"""Drop-in for the reference's envs/my_pong_env_2p.py (PongEnv2P, :10-310).

A PongEnv2P here is a one-arena view of the device environment (pongmi.env.PongEnv2PBatch, the
pm_env_reset / pm_env_step kernels). The scalar API is the reference's:

    env = PongEnv2P(**cfg['env'])            # resets once, like the reference (:81)
    (obsA, obsB) = env.reset()               # f32[7] each
    (obsA, obsB), (rA, rB), done, {} = env.step(aA, aB)

Serves are drawn on the host from the global `random` module with the reference's own draw order
and expressions (:94-110) and handed to the kernel, so a script that seeds `random` sees the
reference's trajectories bit for bit. Each reset() / step() is ONE launch (pm_env_reset1 /
pm_env_step1: actions and serve as kernel arguments, results written straight into a host-mapped
buffer the host polls), with no host-to-device copy, no device-to-host copy and no stream
synchronisation: the same tick as pm_env_step at n = 1, bit for bit. The readable attributes (ball_x, ..., bounce_count) are
fetched from the device on access. render() (:265-306) draws the reference's scene through
pongmi.viewer.ArenaView; pygame is imported lazily, only when enable_render=True.
"""
import ctypes
import random

import numpy as np

from pongmi import _lib
from pongmi.env import PongEnv2PBatch, draw_serve, env_config

_STATE_F64 = ("ball_x", "ball_y", "ball_vx", "ball_vy", "spin", "top_paddle_x", "bottom_paddle_x")
_STATE_I32 = ("scoreA", "scoreB", "bounce_count")


class _Spaces:
    class MultiDiscrete:
        def __init__(self, nvec):
            self.nvec = np.asarray(nvec)

    class Box:
        def __init__(self, low, high, dtype=np.float32):
            self.low, self.high, self.dtype = low, high, dtype
            self.shape = np.asarray(low).shape


class PongEnv2P:
    def __init__(self, render_size=400, paddle_width=0.2, paddle_speed=0.02, max_score=3, enable_render=False,
                 enable_spin=True, magnus_factor=0.01, restitution=0.9, friction=0.2, ball_mass=1.0,
                 world_ball_radius=0.03, ball_speed_range=(0.01, 0.05), spin_range=(-10, 10),
                 ball_angle_intervals=None, speed_scale_every=3, speed_increment=0.2, device="cuda"):
        kw = dict(render_size=render_size, paddle_width=paddle_width, paddle_speed=paddle_speed, max_score=max_score,
                  enable_render=enable_render, enable_spin=enable_spin, magnus_factor=magnus_factor,
                  restitution=restitution, friction=friction, ball_mass=ball_mass,
                  world_ball_radius=world_ball_radius, ball_speed_range=ball_speed_range, spin_range=spin_range,
                  ball_angle_intervals=ball_angle_intervals, speed_scale_every=speed_scale_every,
                  speed_increment=speed_increment)
        self._cfg = env_config(**kw)
        for k, v in self._cfg.items():
            setattr(self, k, v)
        self.spin_angle = 0.0
        self.action_space = _Spaces.MultiDiscrete([3, 3])
        low = np.array([0, 0, -1, -1, 0, 0, -10], dtype=np.float32)
        high = np.array([1, 1, 1, 1, 1, 1, 10], dtype=np.float32)
        self.observation_space = _Spaces.Box(low, high, dtype=np.float32)
        self._env = PongEnv2PBatch(1, device=device, **{k: v for k, v in kw.items()})
        self._lib = _lib.load()
        self._slot = _lib.MappedSlot(18, 17)  # obsA[7] obsB[7] rA rB done | seq
        # per-call constants made once: the argument references, and the launch stream (the one current
        # at construction, held so it outlives every launch; each call waits for its own result, so
        # nothing else orders against it)
        self._pparams, self._pstate = ctypes.byref(self._env.params), ctypes.byref(self._env.state)
        self._stream_ref = _lib.current_stream()
        self._stream = self._stream_ref.cuda_stream
        self._step1, self._reset1 = self._lib.pm_env_step1, self._lib.pm_env_reset1
        self._host = None
        if enable_render:
            import pygame  # noqa: F401  (viewer only; not part of the device path)
        self.reset()

    # ------------------------------------------------------------------ reference API
    def reset(self, seed=None, options=None):
        vx, vy, spin = draw_serve(random, self._cfg)  # 4 draws from the global stream (:94-110)
        self.spin_angle = 0.0
        slot = self._slot
        rc = self._reset1(self._pstate, vx, vy, spin, slot.dev, slot.next_seq(), self._stream)
        if rc:
            _lib.check(rc, "pm_env_reset1")
        self._host = None
        slot.wait()
        out = slot.f32[0:14].copy()
        return out[0:7], out[7:14]

    def step(self, actionA, actionB):
        aA, aB = int(actionA), int(actionB)
        if not (0 <= aA <= 2 and 0 <= aB <= 2):
            raise ValueError(f"actions must be in {{0, 1, 2}}, got ({actionA}, {actionB})")
        slot = self._slot
        rc = self._step1(self._pparams, self._pstate, aA, aB, slot.dev, slot.next_seq(), self._stream)
        if rc:
            _lib.check(rc, "pm_env_step1")
        self._host = None
        slot.wait()
        out = slot.f32[0:17].copy()
        r = out[14:17].tolist()
        return (out[0:7], out[7:14]), (r[0], r[1]), r[2] != 0.0, {}

    def _get_obs(self):
        st = self._state()
        x, y, vx, vy, sp, top, bot = (st[k] for k in _STATE_F64)
        obsA = np.array([x, 1.0 - y, vx, -vy, top, bot, sp], dtype=np.float32)
        obsB = np.array([x, y, vx, vy, bot, top, sp], dtype=np.float32)
        return obsA, obsB

    def render(self):
        """The reference's scene (:265-306) through pongmi.viewer (pygame window; frame() is headless)."""
        if not self.enable_render:
            return
        if getattr(self, "_view", None) is None:
            from pongmi.viewer import ArenaView
            self._view = ArenaView(self._env, 0, self.render_size)
        self._view.spin_angle = self.spin_angle
        self._view.render()
        self.spin_angle = self._view.spin_angle

    def close(self):
        pass

    # ------------------------------------------------------------------ attributes
    def _state(self):
        if self._host is None:
            s = self._env.get_state()
            self._host = {name: s[k] [0] for name, k in zip(_STATE_F64 + _STATE_I32,
                                                             ("x", "y", "vx", "vy", "spin", "top", "bot",
                                                              "scoreA", "scoreB", "bounces"))}
        return self._host

    def __getattr__(self, name):
        if name in _STATE_F64:
            return float(self._state()[name])
        if name in _STATE_I32:
            return int(self._state()[name])
        raise AttributeError(name)
