"""Eager vs graph-replayed vector steps (torch.cuda.CUDAGraph over pm_selfplay_step), same learner.

    python tools/graph_probe.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def main():
    import bench
    from pongmi.selfplay import SelfPlayLearner
    sdB, sdA = bench.synthetic_qnet(1), bench.synthetic_qnet(2)
    pool = [bench.synthetic_qnet(100 + k) for k in range(8)]
    L = SelfPlayLearner(bench.ENV_KW, 65536, sdB, sdA, pool, batch=256, memory_size=1_000_000, epsilon=0.08, seed=7)
    for _ in range(30):
        L.step()
    torch.cuda.synchronize()

    def timeit(fn, reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    print(f"eager: {timeit(L.step, 300) * 1e6:.1f} us/step")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    for per in (1, 10):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            L.step()  # warm on the side stream
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=s):
                for _ in range(per):
                    L.step()
        torch.cuda.synchronize()
        dt = timeit(g.replay, 300 // per) / per
        print(f"graph x{per}: {dt * 1e6:.1f} us/step", flush=True)
    c = L.counters()
    print("counters", c["step"], c["train_steps"], c["epsilon"])


if __name__ == "__main__":
    main()
