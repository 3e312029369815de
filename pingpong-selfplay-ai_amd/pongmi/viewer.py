"""Viewer hook: a PongEnv2P-shaped, read-only view of one arena of device state.

The reference's viewers (tests/test_viewer_v2.py:134-187, tests/pingpong_viewer/**) step their own
PongEnv2P and read ball_x / ball_y / ball_vx / ball_vy / spin / top_paddle_x / bottom_paddle_x /
scoreA / scoreB / paddle_width / world_ball_radius off it. The drop-in envs.my_pong_env_2p.PongEnv2P
already runs them unchanged on a one-arena device batch. ArenaView is the other direction: it looks
at arena `index` of a batch that something else is stepping, such as a PongEnv2PBatch, the self-play
learners or a tournament batch, so a viewer can watch training or a match live. Each refresh() is
one 80-byte device-to-host copy; the arenas stay in HBM.

frame() rasterises what PongEnv2P.render (envs/my_pong_env_2p.py:265-306) draws into an RGB numpy
array: black field, white ball of radius 8 px with the red spin cross, green 10 px paddles. It needs
no pygame, so it can record or test headless. render() blits that frame with pygame when pygame is
installed. The interactive viewer UI (effects, sliders, panels) stays the reference's.
"""
import math

import numpy as np
import torch

_F64 = ("ball_x", "ball_y", "ball_vx", "ball_vy", "spin", "top_paddle_x", "bottom_paddle_x")
_I32 = ("scoreA", "scoreB", "bounce_count")


def _state_of(source):
    """(f64 [7, n], i32 [>=3, n], env config dict) of a batch, a learner, or the drop-in PongEnv2P."""
    inner = getattr(source, "_env", None)
    if inner is not None and hasattr(inner, "f64"):  # envs.my_pong_env_2p.PongEnv2P
        source = inner
    f64, i32 = getattr(source, "f64", None), getattr(source, "i32", None)
    cfg = getattr(source, "env_cfg", None) or getattr(source, "cfg", None)
    if f64 is None or i32 is None or cfg is None:
        raise TypeError("ArenaView needs a PongEnv2PBatch, a self-play learner or a PongEnv2P")
    return f64, i32, dict(cfg)


class ArenaView:
    """Arena `index` of `source` as the attributes a PongEnv2P viewer reads (refresh() to update)."""

    def __init__(self, source, index=0, render_size=None):
        self._f64, self._i32, cfg = _state_of(source)
        n = int(self._f64.shape[1])
        if not 0 <= int(index) < n:
            raise IndexError(f"arena {index} of {n}")
        self.index = int(index)
        self.paddle_width = float(cfg["paddle_width"])
        self.world_ball_radius = float(cfg["world_ball_radius"])
        self.max_score = int(cfg["max_score"])
        self.render_size = int(render_size or cfg.get("render_size", 400))
        self.spin_angle = 0.0  # the reference's render() accumulates it (:281)
        self._screen = None
        self.refresh()

    def refresh(self):
        """Fetch this arena's state: one gather + one device-to-host copy."""
        i = self.index
        row = torch.cat([self._f64[:, i], self._i32[:3, i].to(torch.float64)]).cpu().numpy()
        for k, name in enumerate(_F64):
            setattr(self, name, float(row[k]))
        for k, name in enumerate(_I32):
            setattr(self, name, int(row[7 + k]))
        return self

    def obs(self):
        """(obsA, obsB) float32 as _get_obs_for_A / _get_obs_for_B (:235-257)."""
        x, y, vx, vy, sp, top, bot = (getattr(self, k) for k in _F64)
        return (np.array([x, 1.0 - y, vx, -vy, top, bot, sp], np.float32),
                np.array([x, y, vx, vy, bot, top, sp], np.float32))

    def frame(self, advance_spin=True):
        """RGB uint8 [render_size, render_size, 3] of what render() draws for the current state."""
        if advance_spin:
            self.spin_angle += self.spin
        return draw_frame(self.ball_x, self.ball_y, self.top_paddle_x, self.bottom_paddle_x, self.paddle_width,
                          self.spin_angle, self.render_size)

    def render(self):
        """refresh() + frame() shown in a pygame window (pygame imported on first use)."""
        import pygame
        img = self.refresh().frame()
        if self._screen is None:
            pygame.init()
            self._screen = pygame.display.set_mode((self.render_size, self.render_size))
        for event in pygame.event.get():
            if event.type == pygame.QUIT:
                pygame.quit()
                self._screen = None
                return img
        pygame.surfarray.blit_array(self._screen, img.transpose(1, 0, 2))
        pygame.display.flip()
        return img


def draw_frame(ball_x, ball_y, top_x, bot_x, paddle_width, spin_angle, size):
    """The scene of PongEnv2P.render (:272-302) as an RGB array (no anti-aliasing)."""
    img = np.zeros((size, size, 3), np.uint8)
    bx, by, r = int(ball_x * size), int(ball_y * size), 8
    yy, xx = np.ogrid[:size, :size]
    img[(xx - bx) ** 2 + (yy - by) ** 2 <= r * r] = (255, 255, 255)
    rc = r - 2
    for ang in (spin_angle, spin_angle + 90):
        c, s = math.cos(math.radians(ang)), math.sin(math.radians(ang))
        _line(img, bx + rc * c, by + rc * s, bx - rc * c, by - rc * s, (255, 0, 0))
    pw = int(paddle_width * size)
    for px, y0 in ((int(top_x * size), 0), (int(bot_x * size), size - 10)):
        x0 = px - pw // 2
        img[max(y0, 0):max(min(y0 + 10, size), 0), max(x0, 0):max(min(x0 + pw, size), 0)] = (0, 255, 0)
    return img


def _line(img, x1, y1, x2, y2, color, width=2):
    n = int(max(abs(x2 - x1), abs(y2 - y1))) + 1
    xs = np.rint(np.linspace(x1, x2, n)).astype(int)
    ys = np.rint(np.linspace(y1, y2, n)).astype(int)
    h, w = img.shape[:2]
    for d in range(width):
        ok = (xs + d >= 0) & (xs + d < w) & (ys >= 0) & (ys < h)
        img[ys[ok], xs[ok] + d] = color


def watch(learner, index=0, steps=1000, every=1):
    """Step a self-play learner and yield an ArenaView of arena `index` every `every` vector steps."""
    view = ArenaView(learner, index)
    for t in range(int(steps)):
        learner.step()
        if (t + 1) % every == 0:
            yield view.refresh()
