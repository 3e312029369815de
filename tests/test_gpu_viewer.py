"""Viewer hook on the device: ArenaView follows one arena of a running self-play learner (watch())
and of the drop-in PongEnv2P, reading the same values the batch holds."""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV_KW = dict(paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_spin=True, magnus_factor=0.025, restitution=1,
              friction=0.6, ball_mass=1.0, world_ball_radius=0.03, ball_speed_range=[0.03, 0.05], spin_range=[-5, 5],
              ball_angle_intervals=[[-60, -30], [30, 60]], speed_scale_every=1, speed_increment=0.1)


def test_watch_follows_learner_arena():
    from models.qnet import QNet
    from pongmi.selfplay import SelfPlayLearner
    from pongmi.viewer import watch
    torch.manual_seed(0)
    L = SelfPlayLearner(ENV_KW, 1024, QNet(7, 3).state_dict(), batch=64, memory_size=1 << 14, seed=1)
    seen = []
    for v in watch(L, index=777, steps=40, every=4):
        f, i = L.f64[:, 777].cpu().numpy(), L.i32[:, 777].cpu().numpy()
        assert (v.ball_x, v.ball_y, v.spin, v.top_paddle_x, v.bottom_paddle_x) == (f[0], f[1], f[4], f[5], f[6])
        assert (v.scoreA, v.scoreB, v.bounce_count) == tuple(int(x) for x in i[:3])
        assert np.array_equal(v.obs()[1], L.obsB[777].cpu().numpy())  # the obs the next act reads
        seen.append(v.frame().sum())
    assert len(seen) == 10 and all(s > 0 for s in seen)


def test_view_of_dropin_env_matches_its_attributes():
    from envs.my_pong_env_2p import PongEnv2P
    from pongmi.viewer import ArenaView
    random.seed(4)
    env = PongEnv2P(**ENV_KW)
    v = ArenaView(env)
    for t in range(30):
        (oA, oB), _, done, _ = env.step(t % 3, (t + 1) % 3)
        v.refresh()
        assert (v.ball_x, v.ball_y, v.scoreA, v.bounce_count) == (env.ball_x, env.ball_y, env.scoreA, env.bounce_count)
        assert np.array_equal(v.obs()[0], oA) and np.array_equal(v.obs()[1], oB)
        if done:
            break
