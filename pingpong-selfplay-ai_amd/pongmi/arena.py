"""The persistent model arena (tests/arena.py) on the batched match runner.

The JSON database keeps the reference's format: {"models": [{id, type, path, description}, ...],
"match_history": [{p1, p2, winner, p1_score, p2_score, timestamp}, ...]} (:128-157, :306-313).
A run registers new candidates, plans for every pair (registration order, itertools.combinations)
the episodes still missing towards `episodes_per_match` (pairs counted unordered, :222-244), plays
the whole plan at once through pongmi.tournament.play_matches (serves from the global `random`
stream in the reference's plan order), appends the records in plan order and writes the database
once (the reference rewrites it after every episode). The report is the reference's summary
(:316-351, indexed by model_id).
"""
import json
from datetime import datetime
from pathlib import Path

from .tournament import load_model_universal, play_matches, summarize


def load_database(db_path):
    """The database, or a fresh one when missing / empty / malformed (:128-140)."""
    db_path = Path(db_path)
    if db_path.exists() and db_path.stat().st_size > 0:
        try:
            with open(db_path, "r", encoding="utf-8") as f:
                data = json.load(f)
            data.setdefault("models", [])
            data.setdefault("match_history", [])
            return data
        except json.JSONDecodeError:
            print(f"[warning] database {db_path} is malformed; starting a new one")
    return {"models": [], "match_history": []}


def save_database(db_path, data):
    with open(Path(db_path), "w", encoding="utf-8") as f:
        json.dump(data, f, indent=2, ensure_ascii=False)


def register_models(database, candidates):
    """Append candidates whose id is new; True when any was added (:147-157)."""
    known = {m["id"] for m in database["models"]}
    added = False
    for c in candidates:
        if c["id"] not in known:
            database["models"].append(c)
            known.add(c["id"])
            added = True
    return added


def create_match_plan(database, episodes_per_match):
    """[{p1_id, p2_id, episodes_to_run}] for the pairs short of episodes_per_match (:222-244)."""
    import itertools
    from collections import Counter
    ids = [m["id"] for m in database["models"]]
    played = Counter(tuple(sorted((r["p1"], r["p2"]))) for r in database["match_history"])
    plan = []
    for p1, p2 in itertools.combinations(ids, 2):
        todo = episodes_per_match - played[tuple(sorted((p1, p2)))]
        if todo > 0:
            plan.append({"p1_id": p1, "p2_id": p2, "episodes_to_run": todo})
    return plan


def run_arena(env_params, database, db_path, match_plan, rnn_arch_params, device="cuda", rng=None):
    """Play the plan (matches with a model that fails to load are skipped, :265-283), append the
    records, save the database. Returns the number of episodes played."""
    if not match_plan:
        return 0
    info = {m["id"]: m for m in database["models"]}
    active = {p["p1_id"] for p in match_plan} | {p["p2_id"] for p in match_plan}
    models = {}
    for mid in [m["id"] for m in database["models"] if m["id"] in active]:
        try:
            models[mid] = (load_model_universal({**info[mid], "name": mid}, rnn_arch_params, device), info[mid]["type"])
        except Exception as e:
            print(f"  [error] loading '{mid}' failed: {e}")
    plan = [(p["p1_id"], p["p2_id"], p["episodes_to_run"]) for p in match_plan
            if p["p1_id"] in models and p["p2_id"] in models]
    played = play_matches(env_params, models, plan, device, rng)
    stamp = datetime.utcnow().isoformat() + "Z"
    for a, b, sA, sB in played:
        winner = a if sA > sB else b if sB > sA else "draw"
        database["match_history"].append({"p1": a, "p2": b, "winner": winner, "p1_score": sA, "p2_score": sB,
                                          "timestamp": stamp})
    save_database(db_path, database)
    return len(played)


def generate_summary_report(database):
    """win / lose / draw / games_played / win_rate per model_id over the whole history (:316-351)."""
    ids = [m["id"] for m in database["models"]]
    return summarize([(r["p1"], r["p2"], r["winner"]) for r in database["match_history"]], ids, key="model_id")
