"""The batched round-robin tournament (pongmi.tournament) against the reference's own tournament
loop run on the reference's modules (tests/golden/tournament.npz, make_golden_tournament.py):
5 participants (two QNetRNN checkpoints, a legacy fc.* QNet, a NoisyNet QNet, the ball-follower
bot), 10 pairs x 10 episodes, serves from random.seed(SEED).

Every episode's final (score_A, score_B) must match exactly. (The device and the reference's CPU
torch sum the float32 products in different orders, so a greedy argmax at a near-tie could in
principle flip; none does on these checkpoints and serves, so the test demands every episode.) The
output frames keep the reference's columns.
"""
import random

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV = dict(render_size=400, paddle_width=0.2, paddle_speed=0.03, max_score=3, enable_render=False, enable_spin=True,
           magnus_factor=0.025, restitution=1, friction=0.6, ball_mass=1.0, world_ball_radius=0.03,
           ball_speed_range=[0.03, 0.05], spin_range=[-5, 5], ball_angle_intervals=[[-60, -30], [30, 60]],
           speed_scale_every=1, speed_increment=0.1)  # config.yaml env, as the reference tournament loads it
CKPT_KEY = {"RNN_Gen1": "modelB_state", "RNN_Soul3": "modelB_state", "Legacy4_12": "modelB", "Noisy5_5": "modelB"}


def _write_checkpoints(golden, tmp_path):
    g, gr = golden("tournament"), golden("rnn")
    infos = []
    for i, (name, typ) in enumerate(zip(g["names"].tolist(), g["types"].tolist())):
        if typ == "HardcodedBallFollower":
            infos.append({"name": name, "path": "N/A", "type": typ})
            continue
        if name == "RNN_Soul3":
            sd = {k[7:]: torch.from_numpy(v) for k, v in gr.items() if k.startswith("params.")}
        else:
            sd = {k[len(f"sd{i}."):]: torch.from_numpy(v) for k, v in g.items() if k.startswith(f"sd{i}.")}
        path = tmp_path / f"{name}.pth"
        torch.save({CKPT_KEY[name]: sd, "epsilon": 0.05}, path)
        infos.append({"name": name, "path": str(path), "type": typ})
    return g, infos


def test_tournament_matches_reference_episodes(golden, tmp_path):
    from pongmi.tournament import run_round_robin_tournament
    g, infos = _write_checkpoints(golden, tmp_path)
    E = int(g["scores"].shape[1])
    rng = random.Random(int(g["seed"]))
    match_df, summary_df = run_round_robin_tournament(ENV, {}, infos, E, device="cuda", rng=rng)
    assert rng.random() == float(g["random_state_after"])  # the same draws from the stream
    assert list(match_df.columns) == ["episode", "player_A_name", "player_B_name", "player_A_type", "player_B_type",
                                      "score_A", "score_B", "winner_name"]
    names = g["names"].tolist()
    pairs = g["pairs"].tolist()
    got = match_df[["score_A", "score_B"]].to_numpy().reshape(len(pairs), E, 2)
    assert match_df["player_A_name"].tolist() == [names[i] for i, _ in pairs for _ in range(E)]
    agree = (got == g["scores"]).all(axis=2)
    assert agree.all(), f"{(~agree).sum()} of {agree.size} episodes differ from the reference"
    assert list(summary_df.columns) == ["win", "lose", "draw", "games_played", "win_rate"]
    assert summary_df.index.name == "name" and (summary_df["games_played"] == E * (len(names) - 1)).all()
    assert summary_df["win_rate"].is_monotonic_decreasing
    wins = {nm: 0 for nm in names}
    for p, (i, j) in enumerate(pairs):
        s = g["scores"][p]
        wins[names[i]] += int((s[:, 0] > s[:, 1]).sum())
        wins[names[j]] += int((s[:, 1] > s[:, 0]).sum())
    ref_rates = {nm: w / (E * (len(names) - 1)) for nm, w in wins.items()}
    for nm in names:
        assert summary_df.loc[nm, "win_rate"] == ref_rates[nm], nm


def test_tournament_skips_unloadable_and_writes_csvs(golden, tmp_path):
    from pongmi.tournament import run_round_robin_tournament, save_results
    g, infos = _write_checkpoints(golden, tmp_path)
    infos = infos[2:] + [{"name": "missing", "path": str(tmp_path / "nope.pth"), "type": "QNet"}]
    match_df, summary_df = run_round_robin_tournament(ENV, {}, infos, 4, rng=random.Random(1))
    assert "missing" not in summary_df.index and len(summary_df) == 3 and len(match_df) == 3 * 4
    m, s = save_results(match_df, summary_df, tmp_path / "out", "20250101_000000")
    import pandas as pd
    back = pd.read_csv(s, index_col=0)
    assert list(back.columns) == ["win", "lose", "draw", "games_played", "win_rate"]
    assert pd.read_csv(m)["winner_name"].isin(list(summary_df.index) + ["draw"]).all()


def test_arena_runs_only_missing_episodes(golden, tmp_path):
    """pongmi.arena (tests/arena.py): register -> plan -> batched run -> database; a second run with a
    higher target plays only the missing episodes of each pair."""
    from pongmi.arena import create_match_plan, generate_summary_report, load_database, register_models, run_arena
    _, infos = _write_checkpoints(golden, tmp_path)
    cands = [{"id": i["name"], "type": i["type"], "path": i["path"], "description": ""} for i in infos[2:]]
    db_path = tmp_path / "arena_database.json"
    db = load_database(db_path)
    assert register_models(db, cands)
    assert run_arena(ENV, db, db_path, create_match_plan(db, 6), {}, rng=random.Random(3)) == 3 * 6
    db = load_database(db_path)
    assert len(db["match_history"]) == 18 and create_match_plan(db, 6) == []
    plan = create_match_plan(db, 8)
    assert [p["episodes_to_run"] for p in plan] == [2, 2, 2]
    assert run_arena(ENV, db, db_path, plan, {}, rng=random.Random(4)) == 6
    db = load_database(db_path)
    rep = generate_summary_report(db)
    assert (rep["games_played"] == 16).all() and rep["win"].sum() + rep["draw"].sum() // 2 == 24
    for r in db["match_history"]:
        assert r["winner"] in (r["p1"], r["p2"], "draw") and max(r["p1_score"], r["p2_score"]) == 3
