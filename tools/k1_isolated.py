"""K1 (pm_env_step at 65 536 arenas, autoreset 'done') launched in isolation, for rocprofv3's kernel
trace: under the tracer, back-to-back dispatches are recorded with the tracer's own launch period as
their duration (an empty kernel records 4.46 us mean, profiles/r5_k1_experiments.txt), so this script
separates K1's launches so that each recorded duration is the kernel's own.

    rocprofv3 --kernel-trace --stats --output-format csv -d <dir> -o k -- python tools/k1_isolated.py [mode]

mode "sync" (default): a host synchronize after every launch; mode "spin": a ~20 us spin kernel
(torch.cuda._sleep) in front of every launch on the same stream, no host round trip (the clocks stay
up). 400 launches after 100 warm-up launches back to back.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402,F401  (sys.path for pongmi)
import torch  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "sync"
    from pongmi.env import PongEnv2PBatch
    n = 65536
    env = PongEnv2PBatch(n, seed=3, autoreset="done", **bench.ENV_KW)
    env.reset()
    gen = torch.Generator(device="cuda").manual_seed(0)
    aA = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=gen)
    aB = torch.randint(0, 3, (n,), device="cuda", dtype=torch.int8, generator=gen)
    for _ in range(100):
        env.step(aA, aB)
    torch.cuda.synchronize()
    for _ in range(400):
        if mode == "spin":
            torch.cuda._sleep(40000)
        env.step(aA, aB)
        if mode == "sync":
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    print("k1_isolated done", mode, flush=True)


if __name__ == "__main__":
    main()
