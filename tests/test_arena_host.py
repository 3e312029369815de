"""The arena database logic (pongmi.arena, tests/arena.py) without a GPU: the reference's own
database (tests/golden/arena.npz) reproduces the summary the reference wrote from it, exactly;
registration, plans (unordered pair counts) and the JSON round trip."""
import numpy as np


def _reference_db(golden):
    g = golden("arena")
    ids = g["ids"].tolist()
    models = [{"id": i, "type": t, "path": p, "description": d}
              for i, t, p, d in zip(ids, g["types"].tolist(), g["paths"].tolist(), g["descriptions"].tolist())]
    hist = [{"p1": ids[a], "p2": ids[b], "winner": "draw" if w < 0 else ids[w], "p1_score": int(s1),
             "p2_score": int(s2), "timestamp": "2025-08-06T00:00:00Z"}
            for a, b, w, s1, s2 in zip(g["p1"], g["p2"], g["winner"], g["p1_score"], g["p2_score"])]
    return {"models": models, "match_history": hist}, g


def test_summary_matches_reference_report(golden):
    from pongmi.arena import generate_summary_report
    db, g = _reference_db(golden)
    df = generate_summary_report(db)
    assert df.index.name == "model_id" and list(df.columns) == ["win", "lose", "draw", "games_played", "win_rate"]
    assert df.index.tolist() == g["summary_ids"].tolist()
    for col in ("win", "lose", "draw", "games_played"):
        assert df[col].tolist() == g[f"summary_{col}"].tolist(), col
    np.testing.assert_array_equal(df["win_rate"].to_numpy(), g["summary_win_rate"])


def test_plan_register_roundtrip(golden, tmp_path):
    from pongmi.arena import create_match_plan, load_database, register_models, save_database
    db, _ = _reference_db(golden)
    assert create_match_plan(db, 100) == []  # 45 pairs x 100 played
    plan = create_match_plan(db, 120)
    assert len(plan) == 45 and all(p["episodes_to_run"] == 20 for p in plan)
    assert not register_models(db, [{"id": "RNN_Gen1", "type": "QNetRNN", "path": "x"}])
    assert register_models(db, [{"id": "new", "type": "QNet", "path": "y"}])
    plan = create_match_plan(db, 100)
    assert len(plan) == 10 and all(p["p2_id"] == "new" and p["episodes_to_run"] == 100 for p in plan)
    # pairs count unordered: a record stored as (p2, p1) counts for (p1, p2)
    db["match_history"].append({"p1": "new", "p2": "model2-0", "winner": "new", "p1_score": 3, "p2_score": 0,
                                "timestamp": "t"})
    assert [p["episodes_to_run"] for p in create_match_plan(db, 100) if p["p1_id"] == "model2-0"] == [99]
    path = tmp_path / "arena_database.json"
    save_database(path, db)
    assert load_database(path) == db
    (tmp_path / "bad.json").write_text("{not json")
    assert load_database(tmp_path / "bad.json") == {"models": [], "match_history": []}
    assert load_database(tmp_path / "missing.json") == {"models": [], "match_history": []}


def test_play_plan_blocks_groups_pairs():
    """pongmi.play.plan_blocks: arenas grouped by (net A, net B) in first-appearance order, ascending
    within a pair, each group split into block ranges of per_block slots."""
    import numpy as np
    from pongmi.play import COLUMNS, MAX_SLOTS, TARGET_BLOCKS, plan_blocks
    blk, rng_, order = plan_blocks([0, 1, 0, 1, 0], [2, 2, 2, 2, 2])
    assert blk.tolist() == [[0, 2], [1, 2]] and rng_.tolist() == [[0, 3], [3, 2]] and order.tolist() == [0, 2, 4, 1, 3]
    r = np.random.default_rng(0)
    a, b = r.integers(-1, 3, 1000), r.integers(-1, 3, 1000)
    for per_block in (None, 7, 128):
        blk, rng_, order = plan_blocks(a, b, per_block)
        assert sorted(order.tolist()) == list(range(1000))
        assert rng_[:, 1].sum() == 1000 and (rng_[1:, 0] == np.cumsum(rng_[:, 1])[:-1]).all()
        for (na, nb), (s0, c) in zip(blk, rng_):
            idx = order[s0:s0 + c]
            assert 0 < c <= (per_block or COLUMNS)
            assert (a[idx] == na).all() and (b[idx] == nb).all() and (np.diff(idx) > 0).all()
    big = plan_blocks(np.zeros(COLUMNS * TARGET_BLOCKS * 3), np.ones(COLUMNS * TARGET_BLOCKS * 3))
    assert big[0].shape[0] == TARGET_BLOCKS and (big[1][:, 1] == 3 * COLUMNS).all()
    huge = plan_blocks(np.zeros(MAX_SLOTS * TARGET_BLOCKS * 2), np.ones(MAX_SLOTS * TARGET_BLOCKS * 2))
    assert huge[0].shape[0] == 2 * TARGET_BLOCKS and (huge[1][:, 1] == MAX_SLOTS).all()
    assert plan_blocks([], [])[0].shape == (0, 2)
