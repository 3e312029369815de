"""Statistical replication of the reference's own tournament result with the batched evaluator.

The reference ran tests/test_round_robin.py with six QNetRNN checkpoints and the ball-follower bot,
100 episodes per pair, on config.yaml's env (results/match_records_20250806_213819.csv and
summary_ranking_20250806_213819.csv; their counts are restated below). This replays the same
tournament with pongmi.tournament at `--episodes` per pair (weights from
tests/golden/_local/tournament_models.npz, made by tools/extract_tournament_weights.py) and prints
per-pair and per-model win rates beside the reference's with the two-sample z score. Serves are
random draws, so the comparison is statistical.

    python tools/tournament_replication.py [--episodes 1000]
"""
import argparse
import os
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

ENV = dict(render_size=400, paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_render=False, enable_spin=True,
           magnus_factor=0.025, restitution=1, friction=0.6, ball_mass=1.0, world_ball_radius=0.03,
           ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], ball_angle_intervals=[[-60, -30], [30, 60]],
           speed_scale_every=1, speed_increment=0.1)
NAMES = ["RNN_Gen1", "RNN_Gen2", "RNN_Gen3", "RNN_Gen4", "RNN_Gen5", "RNN_Gen6", "BallFollowerBot"]
# match_records_20250806_213819.csv: (A, B) -> (A wins, B wins) of 100
REF_PAIRS = {
    ("RNN_Gen1", "RNN_Gen2"): (8, 92), ("RNN_Gen1", "RNN_Gen3"): (26, 74), ("RNN_Gen1", "RNN_Gen4"): (14, 86),
    ("RNN_Gen1", "RNN_Gen5"): (29, 71), ("RNN_Gen1", "RNN_Gen6"): (19, 81), ("RNN_Gen1", "BallFollowerBot"): (56, 44),
    ("RNN_Gen2", "RNN_Gen3"): (31, 69), ("RNN_Gen2", "RNN_Gen4"): (32, 68), ("RNN_Gen2", "RNN_Gen5"): (32, 68),
    ("RNN_Gen2", "RNN_Gen6"): (35, 65), ("RNN_Gen2", "BallFollowerBot"): (74, 26), ("RNN_Gen3", "RNN_Gen4"): (33, 67),
    ("RNN_Gen3", "RNN_Gen5"): (50, 50), ("RNN_Gen3", "RNN_Gen6"): (36, 64), ("RNN_Gen3", "BallFollowerBot"): (77, 23),
    ("RNN_Gen4", "RNN_Gen5"): (30, 70), ("RNN_Gen4", "RNN_Gen6"): (31, 69), ("RNN_Gen4", "BallFollowerBot"): (58, 42),
    ("RNN_Gen5", "RNN_Gen6"): (38, 62), ("RNN_Gen5", "BallFollowerBot"): (59, 41),
    ("RNN_Gen6", "BallFollowerBot"): (60, 40),
}
REF_GAMES = 100


def z2(p1, n1, p2, n2):
    p = (p1 * n1 + p2 * n2) / (n1 + n2)
    se = (p * (1 - p) * (1 / n1 + 1 / n2)) ** 0.5
    return 0.0 if se == 0 else (p1 - p2) / se


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    from pongmi.tournament import run_round_robin_tournament
    w = np.load(os.path.join(ROOT, "tests", "golden", "_local", "tournament_models.npz"))
    tmp = tempfile.mkdtemp()
    infos = []
    for nm in NAMES[:-1]:
        sd = {k[len(nm) + 1:]: torch.from_numpy(w[k]) for k in w.files if k.startswith(nm + ".")}
        path = os.path.join(tmp, nm + ".pth")
        torch.save({"modelB_state": sd}, path)
        infos.append({"name": nm, "path": path, "type": "QNetRNN"})
    infos.append({"name": "BallFollowerBot", "path": "N/A", "type": "HardcodedBallFollower"})
    t0 = time.perf_counter()
    match_df, summary_df = run_round_robin_tournament(ENV, {}, infos, a.episodes, rng=random.Random(a.seed))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    E = a.episodes
    print(f"batched tournament: {len(NAMES)} participants, {len(REF_PAIRS)} pairs x {E} episodes "
          f"= {len(match_df)} episodes in {dt:.1f} s (reference: 100 per pair, batch-1)")
    print(f"{'pair':<34} {'ref A win':>9} {'ours A win':>10} {'z':>6}")
    zs = []
    for (A, B), (wa, wb) in REF_PAIRS.items():
        d = match_df[(match_df.player_A_name == A) & (match_df.player_B_name == B)]
        ours = float((d.winner_name == A).mean())
        z = z2(ours, len(d), wa / REF_GAMES, REF_GAMES)
        zs.append(z)
        print(f"{A + ' vs ' + B:<34} {wa / REF_GAMES:9.2f} {ours:10.3f} {z:6.2f}")
    ref_total = {nm: 0 for nm in NAMES}
    for (A, B), (wa, wb) in REF_PAIRS.items():
        ref_total[A] += wa
        ref_total[B] += wb
    print(f"\n{'model':<16} {'ref win_rate':>12} {'ours':>8} {'z':>6}")
    for nm in summary_df.index:
        r = ref_total[nm] / (REF_GAMES * (len(NAMES) - 1))
        o = float(summary_df.loc[nm, "win_rate"])
        print(f"{nm:<16} {r:12.3f} {o:8.3f} {z2(o, E * (len(NAMES) - 1), r, REF_GAMES * (len(NAMES) - 1)):6.2f}")
    zs = np.array(zs)
    print(f"\npair z scores: mean {zs.mean():+.2f}, rms {np.sqrt((zs ** 2).mean()):.2f}, max |z| {np.abs(zs).max():.2f} "
          f"(21 pairs; |z| > 2 expected for ~1 pair by chance)")
    print("ranking (ours):", " > ".join(summary_df.index))


if __name__ == "__main__":
    main()
