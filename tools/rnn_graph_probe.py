"""QNetRNN vector step: eager vs replayed from a HIP graph (µs per step), the bench workload.

    python tools/rnn_graph_probe.py [--steps 200] [--per-graph 10]

The overlapped step flips the opponents' (h, c) double buffer on the host each step, so a graph holds
an even number of steps (it returns to the parity it was captured at). Also checks that the graph
replays the same computation: two learners from the same seed, one eager and one replayed, must end
with bit-identical parameters.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from bench import ENV_KW_RNN, synthetic_rnn  # noqa: E402


def make():
    from pongmi.rnn_selfplay import RNNSelfPlayLearner
    return RNNSelfPlayLearner(ENV_KW_RNN, 32768, synthetic_rnn(1), synthetic_rnn(2),
                              [synthetic_rnn(100 + k) for k in range(4)], epsilon=0.05, seed=7)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--per-graph", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=60)
    a = ap.parse_args()
    G = a.per_graph + (a.per_graph & 1)
    s = torch.cuda.Stream()
    out = {}
    params = {}
    for mode in ("eager", "graph", "eager2"):
        with torch.cuda.stream(s):
            L = make()
            for _ in range(a.warmup):
                L.step()
            torch.cuda.synchronize()
            n = (a.steps // G) * G
            if mode == "graph":
                L.step()  # the side stream and its events exist before capture
                L.step()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):
                    for _ in range(G):
                        L.step()
                torch.cuda.synchronize()
                g.replay()  # first replay outside the timing
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(n // G):
                    g.replay()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                done = a.warmup + 2 + G + n
            else:
                t0 = time.perf_counter()
                for _ in range(n):
                    L.step()
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                done = a.warmup + n
            out[mode] = round((t1 - t0) / n * 1e6, 1)
            # equal step counts for the identity check: run eager learners to the graph learner's count
            params[mode] = (done, L)
    # identity: an eager learner stepped as many times as the graph one must match it bit for bit
    dg, Lg = params["graph"]
    with torch.cuda.stream(s):
        Le = make()
        for _ in range(dg):
            Le.step()
        torch.cuda.synchronize()
    same = bool(torch.equal(Le.learner.params, Lg.learner.params))
    c = Lg.counters()
    print(json.dumps({"us_per_step": out, "per_graph": G, "graph_equals_eager": same,
                      "train_steps": int(c.get("train_steps", c.get("steps", -1))),
                      "status": int(c.get("status", 0))}))


if __name__ == "__main__":
    main()
