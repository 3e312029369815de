#!/usr/bin/env python3
"""Golden fixture for the arena database report (tests/arena.py:128-157, :222-244, :316-351):
the reference's own arena_database.json (models + 4 500 match records) in compact form, and the
summary it produced from that database (results_arena/summary_ranking_20250806_212948.csv).
Run in the build container only:  python -B tests/golden/make_golden_arena.py
"""
import csv
import json
import os

import numpy as np

REF = os.environ.get("PONG_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def main():
    with open(os.path.join(REF, "arena_database.json"), encoding="utf-8") as f:
        db = json.load(f)
    ids = [m["id"] for m in db["models"]]
    idx = {m: k for k, m in enumerate(ids)}
    h = db["match_history"]
    out = {
        "ids": np.array(ids), "types": np.array([m["type"] for m in db["models"]]),
        "paths": np.array([m["path"] for m in db["models"]]),
        "descriptions": np.array([m.get("description", "") for m in db["models"]]),
        "p1": np.array([idx[r["p1"]] for r in h], np.int8), "p2": np.array([idx[r["p2"]] for r in h], np.int8),
        "winner": np.array([-1 if r["winner"] == "draw" else idx[r["winner"]] for r in h], np.int8),
        "p1_score": np.array([r["p1_score"] for r in h], np.int8), "p2_score": np.array([r["p2_score"] for r in h], np.int8),
    }
    with open(os.path.join(REF, "results_arena", "summary_ranking_20250806_212948.csv")) as f:
        rows = list(csv.DictReader(f))
    out["summary_ids"] = np.array([r["model_id"] for r in rows])
    for col in ("win", "lose", "draw", "games_played"):
        out[f"summary_{col}"] = np.array([int(r[col]) for r in rows], np.int64)
    out["summary_win_rate"] = np.array([float(r["win_rate"]) for r in rows])
    np.savez_compressed(os.path.join(OUT, "arena.npz"), **out)
    print("wrote arena.npz", len(h), "records")


if __name__ == "__main__":
    main()
