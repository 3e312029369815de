"""Viewer hook (pongmi.viewer) on the host: ArenaView reads one arena of a batch's SoA state as the
PongEnv2P attributes the reference viewers use (tests/test_viewer_v2.py:134-187), its observations
are _get_obs_for_A/_B (envs/my_pong_env_2p.py:235-257), and frame() draws render()'s scene
(:272-302) headless."""
import numpy as np
import pytest
import torch


class _Batch:
    def __init__(self, n):
        from pongmi.env import env_config
        g = torch.Generator().manual_seed(0)
        self.f64 = torch.rand((7, n), generator=g, dtype=torch.float64)
        self.i32 = torch.randint(0, 3, (4, n), generator=g, dtype=torch.int32)
        self.cfg = env_config(paddle_width=0.2)


def test_arena_view_attributes_and_obs(orc):
    from pongmi.viewer import ArenaView
    b = _Batch(50)
    v = ArenaView(b, 17)
    f, i = b.f64[:, 17].numpy(), b.i32[:, 17].numpy()
    assert (v.ball_x, v.ball_y, v.ball_vx, v.ball_vy, v.spin, v.top_paddle_x, v.bottom_paddle_x) == tuple(f)
    assert (v.scoreA, v.scoreB, v.bounce_count) == tuple(int(x) for x in i[:3])
    assert v.paddle_width == 0.2 and v.render_size == 400 and v.max_score == 3
    arr = np.zeros(1, orc.ARENA_DTYPE)
    for k, name in enumerate(("x", "y", "vx", "vy", "spin", "top", "bot")):
        arr[name] = f[k]
    oA, oB = orc.obs_of_arenas(arr)
    vA, vB = v.obs()
    assert np.array_equal(vA, oA[0]) and np.array_equal(vB, oB[0])
    b.f64[0, 17] = 0.25
    assert v.ball_x != 0.25 and v.refresh().ball_x == 0.25
    with pytest.raises(IndexError):
        ArenaView(b, 50)
    with pytest.raises(TypeError):
        ArenaView(object())


def test_frame_draws_render_scene():
    from pongmi.viewer import draw_frame
    img = draw_frame(0.5, 0.25, 0.3, 0.7, 0.2, 0.0, 400)
    assert img.shape == (400, 400, 3) and img.dtype == np.uint8
    assert tuple(img[103, 204]) == (255, 255, 255)    # ball body (radius 8 at (200, 100)), off the cross
    assert tuple(img[100, 200 + 3]) == (255, 0, 0)    # spin cross at angle 0: horizontal bar
    assert tuple(img[97, 200]) == (255, 0, 0)         # and the vertical one
    assert tuple(img[100, 200 + 10]) == (0, 0, 0)
    assert tuple(img[5, 120]) == (0, 255, 0) and tuple(img[5, 79]) == (0, 0, 0) and tuple(img[10, 120]) == (0, 0, 0)
    assert tuple(img[395, 280]) == (0, 255, 0) and tuple(img[389, 280]) == (0, 0, 0)
    assert (img[:, :, 1] == 255).sum() == 2 * 80 * 10 + (img == 255).all(2).sum()  # paddles + white ball pixels
