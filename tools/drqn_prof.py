"""Back-to-back DRQN updates (B = 64, T = 8, the configs[4] learner) for a kernel-trace profile:

    rocprofv3 --kernel-trace --stats -d gpurun_out/drqn_prof -o drqn -- python3 tools/drqn_prof.py

The product library, the bench's synthetic nets; 20 warm-up updates, then 100 profiled.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pingpong-selfplay-ai_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402


def main():
    import bench
    from pongmi.drqn import DRQNLearner
    B, T = 64, 8
    L = DRQNLearner(bench.synthetic_rnn(1), bench.synthetic_rnn(2), batch=B, T=T)
    g = torch.Generator().manual_seed(0)
    L.load_batch(torch.rand(B, T, 7, generator=g), torch.randint(0, 3, (B, T), generator=g),
                 torch.randint(-1, 2, (B, T), generator=g).float(), torch.rand(B, T, 7, generator=g),
                 torch.rand(B, T, generator=g) < 0.1)
    for _ in range(20):
        L.update()
    torch.cuda.synchronize()
    for _ in range(100):
        L.update()
    torch.cuda.synchronize()
    print("status", L.stats()["status"], "loss", L.stats()["loss"])


if __name__ == "__main__":
    main()
